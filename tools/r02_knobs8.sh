# GPU box: per-rank times of the strong-scaling shards under knob settings (env), first 2 ranks
set -uo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONPATH=.
OUT=gpurun_out/${TAG:-r02_knobs}; mkdir -p $OUT
for cfg in "$@"; do
  echo "== $cfg" >> $OUT/log.txt
  env $cfg timeout -k 10 200 python tools/shard_time.py --ranks 2 ${NS:-4 8} >> $OUT/log.txt 2>&1 || { echo "failed: $cfg"; tail -5 $OUT/log.txt; exit 1; }
done
grep -E "==|N=" $OUT/log.txt
