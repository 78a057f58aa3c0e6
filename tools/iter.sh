# quick iteration: GPU parity tests + bench lines (default accel, then the filtered scan for A/B)
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=.
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 && tail -1 gpurun_out/pytest_gpu.log || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --cpu-baseline 0 > gpurun_out/bench_iter.json 2> gpurun_out/bench_iter.err
cat gpurun_out/bench_iter.json
if [ "${AB:-1}" = "1" ]; then
RTW_ACCEL=1 timeout -k 10 300 python bench.py --steps 2 --warmup 1 --cpu-baseline 0 > gpurun_out/bench_iter_scan.json 2> gpurun_out/bench_iter_scan.err
cat gpurun_out/bench_iter_scan.json
fi
