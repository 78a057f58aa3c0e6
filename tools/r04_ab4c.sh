# Round 4: A/B of library builds with the four counters VERDICT r03 asks for (VALU
# instructions per wave-segment, active-lane fraction, wait share, LDS bank-conflict
# ratio), each build first checked by the parity suite through RTW_LIB.
# Usage: bash tools/r04_ab4c.sh TAG ROUNDS LIB...
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONPATH=.
TAG=$1; ROUNDS=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p $OUT
for L in "$@"; do
  N=$(basename $(dirname $L))
  RTW_LIB=$(realpath $L) timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullframe.py -x -q --timeout 300 --timeout-method thread -k "not config5" > $OUT/pytest_$N.log 2>&1 || { echo "$N: parity FAILED"; tail -30 $OUT/pytest_$N.log; exit 1; }
  echo "$N: $(tail -1 $OUT/pytest_$N.log)"
done
timeout -k 10 900 python -u tools/libab.py $ROUNDS "$@" > $OUT/ab.log 2>&1 || { tail -20 $OUT/ab.log; exit 1; }
tail -${#@} $OUT/ab.log
for L in "$@"; do
  N=$(basename $(dirname $L))
  RTW_LIB=$(realpath $L) timeout -k 10 300 python tools/pmc_diag.py lanes=SQ_INSTS_VALU,SQ_THREAD_CYCLES_VALU,SQ_ACTIVE_INST_VALU,SQ_WAIT_ANY,SQ_WAVE_CYCLES lds=SQ_LDS_BANK_CONFLICT,SQ_LDS_IDX_ACTIVE > $OUT/pmc4_$N.json 2> $OUT/pmc4_$N.err || echo "pmc $N failed"
  python3 - $OUT/pmc4_$N.json $N <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
k = lambda p, c: d[p]["rtw_render_persist"][c]
print(sys.argv[2], "valu_insts", round(k("lanes", "SQ_INSTS_VALU") / 1e9, 2), "e9;",
      "active lanes", round(k("lanes", "SQ_THREAD_CYCLES_VALU") / (64 * k("lanes", "SQ_ACTIVE_INST_VALU")), 3), ";",
      "wait share", round(k("lanes", "SQ_WAIT_ANY") / k("lanes", "SQ_WAVE_CYCLES"), 3), ";",
      "lds conflict ratio", round(k("lds", "SQ_LDS_BANK_CONFLICT") / k("lds", "SQ_LDS_IDX_ACTIVE"), 3))
PY
done
