# Round 4 A/B pass: GPU tests (incl. config 5), the exec-mask microbenchmark, an
# interleaved A/B of library builds, and HBM byte counters (FETCH_SIZE, WRITE_SIZE in
# separate passes) of each build's frame. Usage: bash tools/r04_ab.sh TAG ROUNDS LIB...
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONPATH=.
TAG=$1; ROUNDS=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 120 ./tools/ubench_exec > $OUT/ubench_exec.log 2>&1 || echo "ubench_exec failed"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 900 python -u tools/libab.py $ROUNDS "$@" > $OUT/ab.log 2>&1 || { tail -20 $OUT/ab.log; exit 1; }
tail -${#@} $OUT/ab.log
for L in "$@"; do
  N=$(basename $(dirname $L))
  RTW_LIB=$(realpath $L) timeout -k 10 300 python tools/pmc_diag.py fetch=FETCH_SIZE write=WRITE_SIZE > $OUT/pmc_bytes_$N.json 2> $OUT/pmc_bytes_$N.err || echo "pmc $N failed"
done
cat $OUT/ubench_exec.log
