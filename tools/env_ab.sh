# Interleaved A/B of an environment setting on bench.py (kernel ms), N rounds.
# usage: bash tools/env_ab.sh ROUNDS "ENV_A" "ENV_B" [bench flags...]
set -euo pipefail
R=$1; A=$2; B=$3; shift 3
for i in $(seq 1 $R); do
  for e in "$A" "$B"; do
    ms=$(env $e timeout -k 10 200 python bench.py --cpu-baseline 0 "$@" | python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['roofline']['kernel_ms'])")
    echo "[$e] $ms"
  done
done
