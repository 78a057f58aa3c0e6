set -euo pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=.
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 && tail -1 gpurun_out/pytest_gpu.log || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
bash tools/sweep.sh
if [ "${DIAG:-0}" = "1" ]; then RTW_BUDGET_X=${DIAG_B:-6} timeout -k 10 300 python tools/diag_pix.py 23 > gpurun_out/diag.log 2>&1; grep -E "kernel|timeline|per 10" gpurun_out/diag.log; fi
