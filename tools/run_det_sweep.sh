set -euo pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=.
timeout -k 10 300 python tools/determinism.py > gpurun_out/det.log 2>&1; cat gpurun_out/det.log | grep -v amdgpu.ids
DIAG=1 DIAG_B=10 CFGS="${CFGS:-2:10:64:768:16:1}" bash tools/test_and_sweep.sh
