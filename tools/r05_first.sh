# Round-5 first contact: GPU tests (new group / knob tests), the headline bench with
# its live PMC passes and CPU leg, the fast-mode bench (its roofline must be
# measured now), the one-process group bench, then an interleaved A/B of the
# drain-diet builds (ab/*/librtw.so) at N=1 and the per-rank strong-split times.
# Usage: bash tools/r05_first.sh TAG LIB...
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONPATH=.
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 400 python bench.py --steps 10 > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench.json'));r=d['roofline'];print('N=1', d['ms_per_step'], d['value'], r['frac'], r['pmc_source'][:60], d['cpu_baseline']['runs'])"
timeout -k 10 300 python bench.py --mode fast --steps 10 --cpu-baseline 0 > $OUT/bench_fast.json 2> $OUT/bench_fast.err || { tail -20 $OUT/bench_fast.err; exit 1; }
python3 -c "import json;d=json.load(open('$OUT/bench_fast.json'));r=d['roofline'];print('fast', d['ms_per_step'], d['value'], r['frac'], r['traffic'], r['pmc_source'][:60])"
timeout -k 10 300 python bench.py --gpus 2 --steps 2 --warmup 1 > $OUT/bench_group2.json 2> $OUT/bench_group2.err || { tail -20 $OUT/bench_group2.err; exit 1; }
for L in "$@"; do
  N=$(basename $(dirname $L))
  RTW_LIB=$(realpath $L) timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullframe.py -x -q --timeout 300 --timeout-method thread -k "not config5" > $OUT/pytest_$N.log 2>&1 || { echo "$N: parity FAILED"; tail -30 $OUT/pytest_$N.log; exit 1; }
  echo "$N: $(tail -1 $OUT/pytest_$N.log)"
done
timeout -k 10 900 python -u tools/libab.py 3 "$@" > $OUT/ab.log 2>&1 || { tail -20 $OUT/ab.log; exit 1; }
tail -$# $OUT/ab.log
for L in "$@"; do
  N=$(basename $(dirname $L))
  RTW_LIB=$(realpath $L) timeout -k 10 300 python -u tools/shard_time.py 4 8 > $OUT/shard_time_$N.log 2>&1 || { tail -20 $OUT/shard_time_$N.log; exit 1; }
  echo "== $N"; grep "^N=" $OUT/shard_time_$N.log || tail -5 $OUT/shard_time_$N.log
done
