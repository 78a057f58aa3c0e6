# Round-3 record runs on the GPU box: parity tests, smoke, the bench line (live PMC)
# + its rocprofv3 kernel trace, bench.py lines for configs 3 and 5 (a rank of 8, and
# the whole stress frame on one GPU), config-4 ranks through bench.py --shard-of,
# and every rank of the N=1,2,4,8 splits (tools/shard_time.py).
# Usage: bash tools/configs_r03.sh TAG
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONPATH=.
OUT=gpurun_out/$1
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
timeout -k 10 600 python bench.py --pmc-out $OUT/r03_pmc.json > $OUT/bench.json 2> $OUT/bench.err
cat $OUT/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py --pmc 0 --cpu-baseline 0 --e2e 0 > $OUT/trace.log 2>&1
timeout -k 10 300 python bench.py --samples-sqrt 10 --steps 5 --cpu-baseline 0 --e2e 0 > $OUT/bench_config3.json 2> $OUT/bench_config3.err
timeout -k 10 300 python bench.py --size 4096x2304 --samples-sqrt 45 --shard-of 8:0 --steps 2 --warmup 1 --cpu-baseline 0 --e2e 0 > $OUT/bench_config5_rank0of8.json 2> $OUT/bench_config5.err
timeout -k 10 300 python bench.py --size 4096x2304 --samples-sqrt 45 --steps 1 --warmup 1 --cpu-baseline 0 --e2e 0 --pmc 0 > $OUT/bench_config5_1gpu.json 2>> $OUT/bench_config5.err
for nr in 2:0 4:0 8:0 8:4; do
  timeout -k 10 200 python bench.py --shard-of $nr --steps 3 --warmup 1 --cpu-baseline 0 --e2e 0 > $OUT/bench_config4_rank_${nr/:/of}.json 2>> $OUT/bench_config4.err
done
timeout -k 10 300 python -u tools/shard_time.py 1 2 4 8 > $OUT/shard_time.log 2>&1
cat $OUT/shard_time.log
