set -euo pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=.
mkdir -p gpurun_out
RTW_BUDGET_X=0 timeout -k 10 300 python tools/diag_pix.py 23 > gpurun_out/diag_b0.log 2>&1; cat gpurun_out/diag_b0.log
RTW_BUDGET_X=6 timeout -k 10 300 python tools/diag_pix.py 23 > gpurun_out/diag_b6.log 2>&1; cat gpurun_out/diag_b6.log
RTW_ORDER=0 RTW_BUDGET_X=6 timeout -k 10 300 python tools/diag_pix.py 23 > gpurun_out/diag_b6o0.log 2>&1; cat gpurun_out/diag_b6o0.log
