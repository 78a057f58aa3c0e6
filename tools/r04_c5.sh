# Round 4: the exec-mask microbenchmark, the config-5 GPU tests (whole 4096x2304 s=45
# frame vs the oracle's row sample), and a config-5 bench line with its row parity.
# Usage: bash tools/r04_c5.sh TAG
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONPATH=.
OUT=gpurun_out/${1:-r04_c5}
mkdir -p $OUT
timeout -k 10 120 ./tools/ubench_exec > $OUT/ubench_exec.log 2>&1
cat $OUT/ubench_exec.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_fullframe.py -x -v --timeout 300 --timeout-method thread -k config5 > $OUT/pytest_config5.log 2>&1 || { tail -30 $OUT/pytest_config5.log; exit 1; }
tail -5 $OUT/pytest_config5.log
timeout -k 10 300 python bench.py --size 4096x2304 --samples-sqrt 45 --steps 1 --warmup 1 --pmc 0 --cpu-baseline 0 --e2e 0 > $OUT/bench_config5.json 2> $OUT/bench_config5.err
cat $OUT/bench_config5.json
