# Round-3: knob sweep of strong-scaling shards for several library builds.
# Usage: bash tools/sweep2_r03.sh TAG SHARDS 'SETTINGS' LIB...
set -euo pipefail
cd "$GRAFT_REPO_ROOT"; export PYTHONPATH=. TMPDIR=/tmp
OUT=gpurun_out/$1; SH=$2; SET=$3; shift 3; mkdir -p $OUT
for lib in "$@"; do
  echo "== $lib" >> $OUT/knobs.log
  RTW_LIB=$lib timeout -k 10 600 python -u tools/knob_sweep.py $SH "$SET" 2>&1 | grep -v amdgpu >> $OUT/knobs.log
done
cat $OUT/knobs.log
