# Round 4: heavy-chain latency A/B -- per library build, tools/chain.py on the rows
# whose chains bound the strong split (308: N=8 rank 4 / N=4 rank 0; 455), interleaved
# twice, then the drain stamps of the heavy waves on the diagnostic build.
# Usage: bash tools/r04_chain_ab.sh TAG LIB...
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONPATH=.
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
for rep in 1 2; do
  for L in "$@"; do
    N=$(basename $(dirname $L))
    for ROW in 308 455; do
      echo "== $N row $ROW rep $rep" >> $OUT/chain.log
      CHAIN_ROW=$ROW RTW_LIB=$(realpath $L) timeout -k 10 120 python -u tools/chain.py 2>&1 | grep "^\[" >> $OUT/chain.log
    done
  done
done
cat $OUT/chain.log
RTW_LIB=$(realpath raytracing_in_a_weekend_rust_amd/_lib/librtw_stamps.so) timeout -k 10 120 python -u tools/stamps_drain.py 308 675 1 > $OUT/stamps308.log 2>&1
tail -4 $OUT/stamps308.log
