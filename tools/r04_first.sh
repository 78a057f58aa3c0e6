# Round-4 first contact: GPU tests, the headline bench (no PMC, no CPU leg), the
# one-process group bench on repeated devices, then the fast-mode pass (bench line,
# kernel-trace stats, SQ counters). Usage: bash tools/r04_first.sh TAG [pytest -k expr]
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONPATH=.
OUT=gpurun_out/${1:-r04_first}
K=${2:-}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${K:+-k "$K"} > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python bench.py --steps 5 --pmc 0 --cpu-baseline 0 > $OUT/bench.json 2> $OUT/bench.err
cat $OUT/bench.json
timeout -k 10 300 python bench.py --gpus 2 --steps 2 --warmup 1 > $OUT/bench_group2.json 2> $OUT/bench_group2.err
cat $OUT/bench_group2.json
bash tools/prof_fast.sh ${1:-r04_first}
