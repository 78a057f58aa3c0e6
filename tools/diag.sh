set -euo pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=.
mkdir -p gpurun_out
timeout -k 10 300 python tools/diag_pix.py 23 > gpurun_out/diag.log 2>&1; grep -E "kernel|timeline|per 10|heaviest" gpurun_out/diag.log
