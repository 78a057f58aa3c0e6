# Round-3 measurement pass on the GPU box: parity tests, smoke, the bench line (live
# PMC passes inside it), then a rocprofv3 kernel-trace of the same bench command
# (no counters in that run). Every GPU step has its own time limit; the chain stops
# at the first failure.  Usage: bash tools/prof_r03.sh TAG [pytest-args...]
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONPATH=.
TAG=${1:-run}
shift || true
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "$@" > $OUT/pytest_gpu.log 2>&1 || { tail -60 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
cat $OUT/smoke.log
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err
cat $OUT/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py --pmc 0 --cpu-baseline 0 --e2e 0 > $OUT/trace.log 2>&1
echo "trace done"
