# GPU iteration: parity tests, then knob A/B on shards (tools/knob_sweep.py), then the N=1 tail timeline
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONPATH=.
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 && tail -1 gpurun_out/pytest_gpu.log || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
timeout -k 10 400 python tools/knob_sweep.py "${SHARDS:-1:0,4:0,8:0}" "${KNOBS:-;RTW_INSIDE=0}" > gpurun_out/knob.log 2>&1
cat gpurun_out/knob.log
if [ "${DIAG:-1}" = "1" ]; then
timeout -k 10 200 python tools/diag_pix.py 23 ${DIAG_SHARD:-1 0} > gpurun_out/diag_pix.log 2>&1
cat gpurun_out/diag_pix.log
fi
