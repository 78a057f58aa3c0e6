# Round-3 A/B on the GPU box: parity tests, then interleaved library A/B (bench kernel
# ms at N=1), per-rank times of the strong split, WRITE_SIZE calibration.
# Usage: bash tools/ab_r03.sh TAG ROUNDS LIB...
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONPATH=.
TAG=$1; ROUNDS=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 900 python -u tools/libab.py $ROUNDS "$@" > $OUT/ab.log 2>&1 || { tail -20 $OUT/ab.log; exit 1; }
tail -$# $OUT/ab.log
timeout -k 10 300 python -u tools/shard_time.py 2 4 8 > $OUT/shard_time.log 2>&1
grep -v amdgpu $OUT/shard_time.log
if [ -x tools/ubench_write ]; then
  timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE -d $OUT/ubw -o run --output-format csv -- tools/ubench_write > $OUT/ubench_write.log 2>&1 || true
  python3 -c "
import sys; sys.path.insert(0, '.')
import bench, json
print(json.dumps({k: v.get('WRITE_SIZE') for k, v in bench.read_counters('$OUT/ubw').items()}))" || true
fi
if [ -n "${KNOBS:-}" ]; then
  TAG=$TAG bash tools/knob_ab.sh ${KNOB_ROUNDS:-3} $KNOBS > $OUT/knob_ab.log 2>&1 || { tail -20 $OUT/knob_ab.log; exit 1; }
  tail -4 $OUT/knob_ab.log
fi
