# Round 4 strong-scaling pass: GPU tests, the drained-segment breakdown (stamps build),
# then per library: the heavy row's chains (tools/chain.py) and every rank of the
# N=1/4/8 splits (tools/shard_time.py), and a short interleaved N=1 A/B.
# Usage: bash tools/r04_strong.sh TAG LIB...
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONPATH=.
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
RTW_LIB=raytracing_in_a_weekend_rust_amd/_lib/librtw_stamps.so timeout -k 10 120 python tools/stamps_drain.py > $OUT/stamps_drain.log 2>&1 || echo "stamps_drain failed"
cat $OUT/stamps_drain.log
for L in "$@"; do
  N=$(basename $(dirname $L))
  RTW_LIB=$(realpath $L) timeout -k 10 120 python tools/chain.py > $OUT/chain_$N.log 2>&1
  RTW_LIB=$(realpath $L) timeout -k 10 300 python tools/shard_time.py 1 4 8 > $OUT/shard_time_$N.log 2>&1
  echo "== $N"; tail -1 $OUT/chain_$N.log; grep "^N=" $OUT/shard_time_$N.log
done
timeout -k 10 600 python -u tools/libab.py 3 "$@" > $OUT/ab.log 2>&1 || { tail -20 $OUT/ab.log; exit 1; }
tail -${#@} $OUT/ab.log
