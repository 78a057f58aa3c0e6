# Round 5: heavy-chain latency per library build -- tools/chain.py on rows 308 and 455
# (the chains that bound the strong split), interleaved twice.
# Usage: bash tools/r05_chain.sh TAG LIB...
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
