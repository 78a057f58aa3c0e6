# VALUBusy of the persistent kernel (rocprof's derived metric: 100 * SQ_ACTIVE_INST_VALU
# * 4 / SIMDs / GRBM_GUI_ACTIVE) from one PMC pass of the bench command; counters only,
# no tracing.  Usage: bash tools/pmc_valubusy.sh TAG
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONPATH=.
OUT=gpurun_out/$1
mkdir -p $OUT
timeout -s KILL 150 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT -d $OUT/pmc_busy -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --cpu-baseline 0 > $OUT/pmc_busy.log 2>&1
python3 tools/pmc_insts.py $OUT pmc_busy > $OUT/pmc_busy.json
cat $OUT/pmc_busy.json
