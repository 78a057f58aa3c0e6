# Round-5 A/B of library builds: GPU tests of the tree's build, then interleaved
# N=1 bench rounds, WRITE_SIZE per kernel and the strong-split ranks per build.
# Usage: bash tools/r05_ab.sh TAG ROUNDS SPEC...   (SPEC = ab/x/librtw.so[@ENV=V,...])
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONPATH=.
TAG=$1; ROUNDS=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p $OUT
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
  tail -1 $OUT/pytest_gpu.log
fi
timeout -k 10 1200 python -u tools/libab.py $ROUNDS "$@" > $OUT/ab.log 2>&1 || { tail -20 $OUT/ab.log; exit 1; }
tail -$# $OUT/ab.log
for S in "$@"; do
  L=${S%%@*}; E=""; [ "$S" != "$L" ] && E=${S#*@}
  N=$(basename $(dirname $L))${E:+_${E//[,=]/_}}
  env ${E//,/ } RTW_LIB=$(realpath $L) timeout -k 10 300 python tools/pmc_diag.py ${PMC_MODE:+--mode $PMC_MODE} write=WRITE_SIZE > $OUT/pmc_write_$N.json 2> $OUT/pmc_write_$N.err || echo "pmc $N failed"
  python3 -c "import json,sys;d=json.load(open('$OUT/pmc_write_$N.json'))['write'];print('$N', {k:round(v['WRITE_SIZE']*1024/1e6,1) for k,v in d.items() if v.get('WRITE_SIZE',0)>100})" || true
  if [ "${PMC_INSTS:-0}" = 1 ]; then
    env ${E//,/ } RTW_LIB=$(realpath $L) timeout -k 10 300 python tools/pmc_diag.py insts=SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_LDS,SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_ACTIVE_INST_VALU,SQ_THREAD_CYCLES_VALU > $OUT/pmc_insts_$N.json 2> $OUT/pmc_insts_$N.err || echo "pmc insts $N failed"
    python3 -c "import json;d=json.load(open('$OUT/pmc_insts_$N.json'))['insts']['rtw_render_persist'];print('$N', 'valu %.3fe9 salu %.3fe9 lds %.3fe9 wait %.4f lanes %.4f' % (d['SQ_INSTS_VALU']/1e9, d['SQ_INSTS_SALU']/1e9, d['SQ_INSTS_LDS']/1e9, d['SQ_WAIT_ANY']/d['SQ_WAVE_CYCLES'], d['SQ_THREAD_CYCLES_VALU']/(64*d['SQ_ACTIVE_INST_VALU'])))" || true
  fi
  if [ "${STRONG:-1}" = 1 ]; then
    env ${E//,/ } RTW_LIB=$(realpath $L) timeout -k 10 300 python -u tools/shard_time.py 4 8 > $OUT/shard_time_$N.log 2>&1 || { tail -20 $OUT/shard_time_$N.log; exit 1; }
    grep "^N=" $OUT/shard_time_$N.log | sed "s/^/$N /"
  fi
done
