# Calibrates rocprof's VALUBusy counters (SQ_ACTIVE_INST_VALU, GRBM_GUI_ACTIVE) on the
# VALU microbenchmark, whose kernels run at a known issue rate (tools/ubench_valu.hip).
# Usage: bash tools/pmc_ubench_busy.sh TAG  (ab/ubench_valu built beforehand: hipcc -O3 --offload-arch=gfx950 tools/ubench_valu.hip)
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=gpurun_out/$1
mkdir -p $OUT
timeout -k 10 60 ./ab/ubench_valu > $OUT/ubench.log 2>&1
cat $OUT/ubench.log
timeout -s KILL 90 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $OUT/pmc_ub -o run --output-format csv -- ./ab/ubench_valu > $OUT/pmc_ub.log 2>&1
for k in k_fma32 k_pkfma "k_f64<0>" "k_f64<2>" k_sqrtdiv; do echo "== $k"; python3 tools/pmc_insts.py $OUT pmc_ub "$k"; done > $OUT/pmc_ub.json
cat $OUT/pmc_ub.json
