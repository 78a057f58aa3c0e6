# Round-3: interleaved A/B of library builds on one rank of a strong split and at N=1.
# Usage: bash tools/ab_shard_r03.sh TAG ROUNDS 'N:r ...' LIB...
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONPATH=.
OUT=gpurun_out/$1; R=$2; SH=$3; shift 3
mkdir -p $OUT
for s in $SH; do
  if [ "$s" = "1:0" ]; then A=""; else A="--shard-of $s"; fi
  LIBAB_ARGS="$A" timeout -k 10 600 python -u tools/libab.py $R "$@" > $OUT/ab_${s/:/of}.log 2>&1 || { tail -20 $OUT/ab_${s/:/of}.log; exit 1; }
  echo "[$s]"; tail -$# $OUT/ab_${s/:/of}.log
done
