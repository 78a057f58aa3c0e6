# GPU box: rank-0 time of the N=8 row shard under drain-group knobs (strong scaling study)
set -uo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONPATH=.
OUT=gpurun_out/r02_knobs8; mkdir -p $OUT
for cfg in "X=1" "RTW_COOPG=16" "RTW_COOPG=16 RTW_BUDGET_X=2" "RTW_COOPG=64 RTW_BUDGET_X=2" "RTW_COOPG=16 RTW_BUDGET_X=4" "RTW_COOPG=16 RTW_BUDGET_X=3 RTW_RATE_X=6 RTW_RATE_K=8" "RTW_COOPG=64 RTW_BUDGET_X=3 RTW_RATE_X=6 RTW_RATE_K=8"; do
  echo "== $cfg" >> $OUT/log.txt
  env $cfg timeout -k 10 120 python tools/shard_time.py --ranks 1 8 >> $OUT/log.txt 2>&1 || { echo "failed: $cfg"; tail -5 $OUT/log.txt; exit 1; }
done
grep -E "==|N=" $OUT/log.txt
