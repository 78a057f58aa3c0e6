# Round-3 knob sweep (strong-scaling shards) + per-pixel timelines of the N=4/N=8
# ranks. Usage: bash tools/knobs_r03.sh TAG
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONPATH=.
OUT=gpurun_out/$1
mkdir -p $OUT
timeout -k 10 600 python -u tools/knob_sweep.py 1:0,2:0,4:0,8:4 \
  ';RTW_HOT_PRIO=1;RTW_HOT_PRIO=3;RTW_HOT_PRIO=10;RTW_HEAVY=3;RTW_HEAVY=3 RTW_HOT_PRIO=3;RTW_ENDGAME=4500;RTW_ENDGAME=6000;RTW_HEAVY=3 RTW_ENDGAME=6000' \
  > $OUT/knobs.log 2>&1
cat $OUT/knobs.log
timeout -k 10 120 python -u tools/diag_pix.py 23 8 4 > $OUT/diag_n8_r4.log 2>&1
timeout -k 10 120 python -u tools/diag_pix.py 23 4 0 > $OUT/diag_n4_r0.log 2>&1
grep -v amdgpu.ids $OUT/diag_n8_r4.log $OUT/diag_n4_r0.log
