# Round-3 small-shard knob sweep (strong scaling): rate-based parking and priority
# waves at N=4 and N=8 ranks. Usage: bash tools/knobs_r03.sh TAG
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONPATH=.
OUT=gpurun_out/$1
mkdir -p $OUT
timeout -k 10 400 python -u tools/knob_sweep.py 2:0,4:0,8:4 \
  ';RTW_RATE_X=8;RTW_RATE_X=6;RTW_RATE_X=8 RTW_RATE_K=4;RTW_RATE_X=6 RTW_RATE_K=4;RTW_RATE_X=4 RTW_RATE_K=4;RTW_RATE_X=3 RTW_RATE_K=2;RTW_HEAVY=1;RTW_HEAVY=2 RTW_RATE_X=6 RTW_RATE_K=4' \
  > $OUT/knobs.log 2>&1
cat $OUT/knobs.log
