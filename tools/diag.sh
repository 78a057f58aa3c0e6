set -euo pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=.
mkdir -p gpurun_out
RTW_PERSIST=0 RTW_BUDGET_X=0 RTW_LIB=$PWD/raytracing_in_a_weekend_rust_amd/_lib/librtw_stamps.so RTW_ACCEL=2 timeout -k 10 300 python tools/stamps.py 10 > gpurun_out/stamps_bvh4.log 2>&1; cat gpurun_out/stamps_bvh4.log
