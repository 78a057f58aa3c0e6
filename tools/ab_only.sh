set -euo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONPATH=.
mkdir -p gpurun_out/$1
timeout -k 10 600 python -u tools/libab.py $2 ${@:3} > gpurun_out/$1/ab.log 2>&1 || { tail -20 gpurun_out/$1/ab.log; exit 1; }
tail -$(( $# - 2 )) gpurun_out/$1/ab.log
