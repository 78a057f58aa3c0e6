set -euo pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=. RTW_COOPG=64 RTW_HEAVY=2
for rk in 16 8 4; do
  for rx in 16 20; do
    RTW_RATE_K=$rk RTW_RATE_X=$rx timeout -k 10 120 python bench.py --steps 3 --warmup 1 --cpu-baseline 0 > gpurun_out/rk.json 2>/dev/null
    python3 -c "import json;d=json.load(open('gpurun_out/rk.json'));print('rate_k $rk rate_x $rx', d['ms_per_step'], d['stats']['parked_pixels'])"
  done
done
