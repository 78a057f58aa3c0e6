# Fast-mode measurement pass on the GPU box: bench line, kernel-trace stats, and
# one PMC pass (SQ counters only, no tracing). Usage: bash tools/prof_fast.sh TAG
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONPATH=.
OUT=gpurun_out/${1:-fast}
mkdir -p $OUT
timeout -k 10 200 python bench.py --mode fast --cpu-baseline 0 > $OUT/bench_fast.json 2> $OUT/bench_fast.err
cat $OUT/bench_fast.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace_fast -o run --output-format csv -- python3 bench.py --mode fast --cpu-baseline 0 > $OUT/trace_fast.log 2>&1
echo "trace done"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU -d $OUT/pmc_fast -o run --output-format csv -- python3 bench.py --mode fast --steps 1 --warmup 0 --cpu-baseline 0 > $OUT/pmc_fast.log 2>&1
python3 tools/pmc_insts.py $OUT pmc_fast rtw_fast_render > $OUT/pmc_fast.json || true
cat $OUT/pmc_fast.json || true
