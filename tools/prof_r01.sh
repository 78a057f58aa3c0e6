# Round-1 profiling: bench JSON, rocprofv3 kernel-trace stats of the bench
# command, then separate PMC passes (counters never combined with tracing).
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONPATH=.
OUT=gpurun_out/r01
mkdir -p $OUT
timeout -k 10 300 python bench.py --steps 3 --warmup 1 > $OUT/bench.json 2> $OUT/bench.err
echo "bench done"; cat $OUT/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --cpu-baseline 0 > $OUT/trace.log 2>&1
echo "trace done"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $OUT/pmc1 -o run --output-format csv -- python bench.py --steps 1 --warmup 0 --cpu-baseline 0 > $OUT/pmc1.log 2>&1
echo "pmc1 done"
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM -d $OUT/pmc2 -o run --output-format csv -- python bench.py --steps 1 --warmup 0 --cpu-baseline 0 > $OUT/pmc2.log 2>&1
echo "pmc2 done"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc3 -o run --output-format csv -- python bench.py --steps 1 --warmup 0 --cpu-baseline 0 > $OUT/pmc3.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc4 -o run --output-format csv -- python bench.py --steps 1 --warmup 0 --cpu-baseline 0 > $OUT/pmc4.log 2>&1
echo "pmc done"
