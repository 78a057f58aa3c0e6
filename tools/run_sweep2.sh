set -euo pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=.
DIAG=1 DIAG_B=10 CFGS="2:10:64:768:16:1 2:10:64:768:20:1 2:10:64:768:24:1 2:15:64:768:16:1 2:10:64:768:16:2 2:20:64:768:24:1" bash tools/test_and_sweep.sh
