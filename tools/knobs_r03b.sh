# Round-3 knob sweep: 16-lane drain groups with medium-pixel parking.
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONPATH=.
OUT=gpurun_out/$1
mkdir -p $OUT
timeout -k 10 600 python -u tools/knob_sweep.py 2:0,4:0,8:4 \
  ';RTW_COOPG=16;RTW_COOPG=16 RTW_RATE_X=8 RTW_RATE_K=64;RTW_COOPG=16 RTW_RATE_X=10 RTW_RATE_K=32;RTW_COOPG=16 RTW_HEAVY=3 RTW_RATE_X=8 RTW_RATE_K=64;RTW_COOPG=16 RTW_HEAVY=4 RTW_RATE_X=8 RTW_RATE_K=32' \
  > $OUT/knobs.log 2>&1
cat $OUT/knobs.log
