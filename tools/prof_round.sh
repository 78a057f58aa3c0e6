# Full measurement pass on the GPU box: parity tests, smoke, bench JSON (with the
# CPU baseline), rocprofv3 kernel-trace stats of the same bench command, then
# separate PMC passes: HBM bytes (FETCH_SIZE and WRITE_SIZE never share a pass),
# instruction counts (8 SQ counters), and wave cycle counters (last: optional).
# Counters are never combined with tracing.  Usage: bash tools/prof_round.sh TAG
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONPATH=.
TAG=${1:-run}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
cat $OUT/smoke.log
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err
cat $OUT/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py --cpu-baseline 0 > $OUT/trace.log 2>&1
echo "trace done"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --cpu-baseline 0 > $OUT/pmc_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --cpu-baseline 0 > $OUT/pmc_write.log 2>&1
python3 tools/pmc_traffic.py $OUT > $OUT/pmc_traffic.json
cat $OUT/pmc_traffic.json
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_INT64 -d $OUT/pmc_insts -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --cpu-baseline 0 > $OUT/pmc_insts.log 2>&1
python3 tools/pmc_insts.py $OUT pmc_insts > $OUT/pmc_insts.json
cat $OUT/pmc_insts.json
if timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY -d $OUT/pmc_cycles -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --cpu-baseline 0 > $OUT/pmc_cycles.log 2>&1; then
  python3 tools/pmc_insts.py $OUT pmc_cycles > $OUT/pmc_cycles.json
  cat $OUT/pmc_cycles.json
else
  echo "cycle counters pass failed (see pmc_cycles.log)"
fi
