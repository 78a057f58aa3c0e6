# GPU box: interleaved A/B of environment settings on bench.py (kernel ms), N rounds.
# usage: bash tools/knob_ab.sh ROUNDS "ENV_A" "ENV_B" ...   (each ENV a space-separated list)
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONPATH=.
OUT=gpurun_out/${TAG:-knob_ab}; mkdir -p $OUT
R=$1; shift
for i in $(seq 1 $R); do
  for e in "$@"; do
    ms=$(env $e timeout -k 10 200 python bench.py --cpu-baseline 0 --e2e 0 --pmc 0 --steps 3 --warmup 1 | python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['roofline']['kernel_ms'])")
    echo "[$e] $ms" | tee -a $OUT/log.txt
  done
done
python3 - $OUT/log.txt <<'PY'
import sys, collections, re
d = collections.defaultdict(list)
for line in open(sys.argv[1]):
    m = re.match(r"\[(.*)\] ([0-9.]+)", line)
    if m: d[m.group(1)].append(float(m.group(2)))
for k, v in d.items(): print(f"{k:40s} mean {sum(v)/len(v):8.2f}  {v}")
PY
