# Drain-path A/B on the GPU box: GPU parity tests, then the shards of every N under
# the drain knobs.  Usage: bash tools/drain_r03.sh TAG
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONPATH=.
OUT=gpurun_out/$1
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 500 python -u tools/knob_sweep.py 1:0,2:0,4:0,8:4 \
  ';RTW_DRAIN_PRIO=0;RTW_HEAVY=1;RTW_HEAVY=1 RTW_DRAIN_PRIO=0;RTW_HEAVY=2;RTW_PREPARK=40;RTW_PREPARK=60;RTW_PREPARK=40 RTW_HEAVY=1;RTW_PREPARK=60 RTW_HEAVY=1' \
  > $OUT/knobs.log 2>&1
cat $OUT/knobs.log
timeout -k 10 300 python -u tools/libab.py 3 raytracing_in_a_weekend_rust_amd/_lib/librtw.so ab/no_tir_cache/librtw.so > $OUT/ab_tir.log 2>&1
tail -2 $OUT/ab_tir.log
