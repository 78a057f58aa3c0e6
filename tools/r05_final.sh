# Round-5 record pass on the GPU box: GPU tests, smoke, the headline bench line (live
# PMC passes, CPU baseline, end-to-end), rocprofv3 kernel-trace stats of the same
# command, configs 3 and 5, the one-process 2-entry group line, fast mode, and every
# rank of the N=1/2/4/8 strong split. Usage: bash tools/r05_final.sh TAG
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONPATH=.
TAG=${1:-r05_final}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
cat $OUT/smoke.log
timeout -k 10 500 python bench.py --steps 10 --warmup 2 --pmc-out $OUT/pmc.json > $OUT/bench.json 2> $OUT/bench.err
cat $OUT/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --cpu-baseline 0 --pmc 0 --e2e 0 > $OUT/trace.log 2>&1
echo "trace done"
timeout -k 10 400 python bench.py --samples-sqrt 10 --steps 5 > $OUT/bench_config3.json 2> $OUT/bench_config3.err
cat $OUT/bench_config3.json
timeout -k 10 300 python bench.py --size 4096x2304 --samples-sqrt 45 --steps 1 --warmup 1 --cpu-baseline 0 --pmc 0 --e2e 0 > $OUT/bench_config5.json 2> $OUT/bench_config5.err
cat $OUT/bench_config5.json
timeout -k 10 300 python bench.py --gpus 2 --steps 2 --warmup 1 > $OUT/bench_group2.json 2> $OUT/bench_group2.err
cat $OUT/bench_group2.json
timeout -k 10 300 python bench.py --mode fast --steps 5 --cpu-baseline 0 > $OUT/bench_fast.json 2> $OUT/bench_fast.err && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace_fast -o run --output-format csv -- python3 bench.py --mode fast --steps 5 --cpu-baseline 0 --pmc 0 --e2e 0 > $OUT/trace_fast.log 2>&1
cat $OUT/bench_fast.json
timeout -k 10 400 python tools/shard_time.py 1 2 4 8 > $OUT/shard_time.log 2>&1
grep "^N=" $OUT/shard_time.log
timeout -k 10 300 python tools/config12.py > $OUT/config12.json 2>&1
timeout -k 10 300 python bench.py --shard-of 8:4 --steps 3 --cpu-baseline 0 --e2e 0 > $OUT/bench_shard8_4.json 2> $OUT/bench_shard8_4.err
cat $OUT/config12.json
