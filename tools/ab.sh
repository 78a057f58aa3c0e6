# GPU tests, then the sweep once per env variant in $AB (space-separated, "-" = none)
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=.
mkdir -p gpurun_out
if [ "${TESTS:-1}" = "1" ]; then
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 && tail -1 gpurun_out/pytest_gpu.log || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
fi
for v in ${AB:--}; do
  echo "#### variant $v"
  if [ "$v" = "-" ]; then SWEEP_OUT=gpurun_out/sweep_base bash tools/sweep.sh; else env $v SWEEP_OUT=gpurun_out/sweep_$v bash tools/sweep.sh; fi
done
