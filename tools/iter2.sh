# quick iteration: GPU parity tests, a bench line, per-rank shard times (tools/shard_time.py)
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=.
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && tail -1 gpurun_out/pytest_gpu.log || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --cpu-baseline 0 > gpurun_out/bench_iter.json 2> gpurun_out/bench_iter.err
cat gpurun_out/bench_iter.json
if [ "${SHARD:-1}" = "1" ]; then
timeout -k 10 300 python tools/shard_time.py ${SHARD_N:-1 2 4 8} > gpurun_out/shard_time.log 2>&1
cat gpurun_out/shard_time.log
fi
