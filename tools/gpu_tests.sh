set -euo pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export PYTHONPATH=.
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 && echo "pytest ok" || { echo "pytest FAILED"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; cat gpurun_out/smoke.log
(cd gpurun_out && timeout -k 10 120 ../raytracing_in_a_weekend_rust_amd/_lib/rtw_cli -h 225 -w 400 -s 3 --depth 8 --seed 1764892800000 --out cli.ppm > cli.log 2>&1); tail -2 gpurun_out/cli.log
