# GPU box: interleaved A/B of library builds and what each one does to the counters
# (replaces the rounds' one-off wrappers: ab_round/ab_only, r04_ab*, r05_ab, r05_chain).
# Usage: bash tools/ab.sh TAG ROUNDS SPEC...   SPEC = ab/x/librtw.so[@ENV=V,...]
# Steps (environment switches, 0/1):
#   TESTS=1    GPU tests of the tree's own build first
#   PARITY=0   the parity suite (no config 5) through RTW_LIB for every build
#   WRITE=1    WRITE_SIZE per kernel and build (tools/pmc_diag.py)
#   INSTS=0    VALU/SALU/LDS instructions, wait share and active lanes per build
#   STRONG=0   every rank of the N=4 and N=8 strong split per build (tools/shard_time.py)
#   CHAIN=0    heavy-chain latency of rows 308 and 455 per build (tools/chain.py)
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONPATH=.
TAG=$1; ROUNDS=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p $OUT
name_of() {  # ab/x/librtw.so@A=1,B=2 -> x_A_1_B_2
  local L=${1%%@*} E=""; [ "$1" != "$L" ] && E=${1#*@}
  echo "$(basename $(dirname $L))${E:+_${E//[,=]/_}}"
}
env_of() { local L=${1%%@*}; [ "$1" != "$L" ] && echo "${1#*@}" | tr ',' ' ' || true; }
lib_of() { realpath ${1%%@*}; }
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
  tail -1 $OUT/pytest_gpu.log
fi
if [ "${PARITY:-0}" = 1 ]; then
  for S in "$@"; do
    N=$(name_of $S)
    env $(env_of $S) RTW_LIB=$(lib_of $S) timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullframe.py -x -q --timeout 300 --timeout-method thread -k "not config5" > $OUT/pytest_$N.log 2>&1 || { echo "$N: parity FAILED"; tail -30 $OUT/pytest_$N.log; exit 1; }
    echo "$N: $(tail -1 $OUT/pytest_$N.log)"
  done
fi
timeout -k 10 1200 python -u tools/libab.py $ROUNDS "$@" > $OUT/ab.log 2>&1 || { tail -20 $OUT/ab.log; exit 1; }
tail -$# $OUT/ab.log
for S in "$@"; do
  N=$(name_of $S)
  if [ "${WRITE:-1}" = 1 ]; then
    env $(env_of $S) RTW_LIB=$(lib_of $S) timeout -k 10 300 python tools/pmc_diag.py write=WRITE_SIZE > $OUT/pmc_write_$N.json 2> $OUT/pmc_write_$N.err || echo "pmc $N failed"
    python3 -c "import json;d=json.load(open('$OUT/pmc_write_$N.json'))['write'];print('$N write MB', {k:round(v['WRITE_SIZE']*1024/1e6,1) for k,v in d.items() if v.get('WRITE_SIZE',0)>100})" || true
  fi
  if [ "${INSTS:-0}" = 1 ]; then
    env $(env_of $S) RTW_LIB=$(lib_of $S) timeout -k 10 300 python tools/pmc_diag.py insts=SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_LDS,SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_ACTIVE_INST_VALU,SQ_THREAD_CYCLES_VALU > $OUT/pmc_insts_$N.json 2> $OUT/pmc_insts_$N.err || echo "pmc insts $N failed"
    python3 -c "import json;d=json.load(open('$OUT/pmc_insts_$N.json'))['insts']['rtw_render_persist'];print('$N', 'valu %.3fe9 salu %.3fe9 lds %.3fe9 wait %.4f lanes %.4f' % (d['SQ_INSTS_VALU']/1e9, d['SQ_INSTS_SALU']/1e9, d['SQ_INSTS_LDS']/1e9, d['SQ_WAIT_ANY']/d['SQ_WAVE_CYCLES'], d['SQ_THREAD_CYCLES_VALU']/(64*d['SQ_ACTIVE_INST_VALU'])))" || true
  fi
  if [ "${STRONG:-0}" = 1 ]; then
    env $(env_of $S) RTW_LIB=$(lib_of $S) timeout -k 10 300 python -u tools/shard_time.py 4 8 > $OUT/shard_time_$N.log 2>&1 || { tail -20 $OUT/shard_time_$N.log; exit 1; }
    grep "^N=" $OUT/shard_time_$N.log | sed "s/^/$N /"
  fi
  if [ "${CHAIN:-0}" = 1 ]; then
    for ROW in 308 455; do
      echo "== $N row $ROW" >> $OUT/chain.log
      env $(env_of $S) CHAIN_ROW=$ROW RTW_LIB=$(lib_of $S) timeout -k 10 120 python -u tools/chain.py 2>&1 | grep "^\[" >> $OUT/chain.log
    done
  fi
done
[ "${CHAIN:-0}" = 1 ] && cat $OUT/chain.log || true
