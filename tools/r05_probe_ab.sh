# A/B of two library builds plus a rocprofv3 kernel-time summary of each (csv).
# Usage: bash tools/r05_probe_ab.sh TAG ROUNDS LIB_A LIB_B
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONPATH=.
TAG=$1; ROUNDS=$2; A=$3; B=$4
OUT=gpurun_out/$TAG
mkdir -p $OUT
STRONG=0 bash tools/r05_ab.sh $TAG $ROUNDS $A $B
for L in $A $B; do
  N=$(basename $(dirname $L))
  RTW_LIB=$(realpath $L) timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace_$N -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --cpu-baseline 0 --pmc 0 --e2e 0 > $OUT/trace_$N.log 2>&1
  f=$(find $OUT/trace_$N -name "*kernel_stats.csv" | head -1)
  echo "== $N"; grep -E "rtw_cost|rtw_seed|persist" $f | sed 's/(anonymous namespace):://g' | awk -F'",' '{print $1"\" "$2}' | cut -d, -f1-4
done
