# Round-3: parity tests, then a knob sweep of strong-scaling shards (images checked
# against the first setting's). Usage: bash tools/sweep_r03.sh TAG 'SETTINGS'
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONPATH=.
OUT=gpurun_out/$1
mkdir -p $OUT
if [ -z "${NOTEST:-}" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
  tail -1 $OUT/pytest_gpu.log
fi
timeout -k 10 900 python -u tools/knob_sweep.py ${SHARDS:-1:0,2:0,4:0,8:4} "$2" > $OUT/knobs.log 2>&1
grep -v amdgpu.ids $OUT/knobs.log
