set -euo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONPATH=.
OUT=gpurun_out/r05_agg; mkdir -p $OUT
STRONG=0 bash tools/r05_ab.sh r05_agg 4 ab/base/librtw.so ab/agg/librtw.so
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/trace -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 1 --cpu-baseline 0 --pmc 0 --e2e 0 > $GRAFT_REPO_ROOT/$OUT/trace.log 2>&1
cd $GRAFT_REPO_ROOT && find $OUT/trace -name "*kernel_stats.csv" | head -1 | xargs cut -d, -f1-4 | sed 's/(anonymous namespace):://g' | cut -c1-120
