# GPU box: the record pass of a round (replaces the rounds' r0N_final/r0N_first wrappers).
# Usage: bash tools/record.sh TAG [STEP...]
# Steps (default: all of them, in this order):
#   tests     GPU tests (pytest -m gpu) and smoke()
#   bench     the headline bench line (live PMC passes, CPU baseline, end to end) and the
#             rocprofv3 kernel-trace stats of the same command
#   config3   BASELINE configs[2] (s=10)
#   config5   BASELINE configs[4] (4096x2304, s=45) whole frame with live PMC passes
#   config5r  every rank of its 8-way split (--shard-of 8:r) with live PMC passes
#   group2    the one-process 2-entry group line
#   fast      the f32 fast-mode line and its rocprofv3 stats
#   strong    every rank of the N=1/2/4/8 strong split (tools/shard_time.py) and rank 4 of 8
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONPATH=.
TAG=${1:?TAG}; shift
STEPS=${*:-tests bench config3 config5 group2 fast strong}
OUT=gpurun_out/$TAG
mkdir -p $OUT
for step in $STEPS; do
  case $step in
  tests)
    timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
    tail -1 $OUT/pytest_gpu.log
    timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
    cat $OUT/smoke.log ;;
  bench)
    timeout -k 10 500 python bench.py --steps 10 --warmup 2 --pmc-out $OUT/pmc.json > $OUT/bench.json 2> $OUT/bench.err
    cat $OUT/bench.json
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --cpu-baseline 0 --pmc 0 --e2e 0 > $OUT/trace.log 2>&1
    echo "trace done" ;;
  config3)
    timeout -k 10 400 python bench.py --samples-sqrt 10 --steps 5 > $OUT/bench_config3.json 2> $OUT/bench_config3.err
    cat $OUT/bench_config3.json ;;
  config5)
    timeout -k 10 400 python bench.py --size 4096x2304 --samples-sqrt 45 --steps 1 --warmup 1 --cpu-baseline 0 --e2e 0 > $OUT/bench_config5.json 2> $OUT/bench_config5.err
    cat $OUT/bench_config5.json ;;
  config5r)
    for r in 0 1 2 3 4 5 6 7; do
      timeout -k 10 300 python bench.py --size 4096x2304 --samples-sqrt 45 --shard-of 8:$r --steps 1 --warmup 1 --cpu-baseline 0 --e2e 0 > $OUT/bench_config5_rank${r}of8.json 2> $OUT/bench_config5_rank${r}of8.err
      python3 -c "import json;d=json.load(open('$OUT/bench_config5_rank${r}of8.json'));print('rank $r', d['ms_per_step'], 'ms', d['roofline']['frac'], d['roofline'].get('traffic'))"
    done ;;
  group2)
    timeout -k 10 300 python bench.py --gpus 2 --steps 2 --warmup 1 > $OUT/bench_group2.json 2> $OUT/bench_group2.err
    cat $OUT/bench_group2.json ;;
  fast)
    timeout -k 10 300 python bench.py --mode fast --steps 5 --cpu-baseline 0 > $OUT/bench_fast.json 2> $OUT/bench_fast.err
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace_fast -o run --output-format csv -- python3 bench.py --mode fast --steps 5 --cpu-baseline 0 --pmc 0 --e2e 0 > $OUT/trace_fast.log 2>&1
    cat $OUT/bench_fast.json ;;
  strong)
    timeout -k 10 400 python tools/shard_time.py 1 2 4 8 > $OUT/shard_time.log 2>&1
    grep "^N=" $OUT/shard_time.log
    timeout -k 10 300 python bench.py --shard-of 8:4 --steps 3 --cpu-baseline 0 --e2e 0 > $OUT/bench_shard8_4.json 2> $OUT/bench_shard8_4.err
    python3 -c "import json;d=json.load(open('$OUT/bench_shard8_4.json'));print('shard 8:4', d['ms_per_step'], d['roofline']['frac'])" ;;
  *) echo "unknown step $step"; exit 2 ;;
  esac
done
