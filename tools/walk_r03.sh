# Round-3: walker-wave build: parity (full frames + parity suite) on RTW_LIB, then
# interleaved A/B against the default build at N=1 and on strong-split ranks.
# Usage: bash tools/walk_r03.sh TAG LIB
set -euo pipefail
cd "$GRAFT_REPO_ROOT"; export PYTHONPATH=. TMPDIR=/tmp
OUT=gpurun_out/$1; LIB=$2; mkdir -p $OUT
RTW_LIB=$LIB timeout -k 10 300 python -u -m pytest tests/test_gpu_fullframe.py -m gpu -x -q --timeout 120 --timeout-method thread -k "one_shot or multi4" > $OUT/ff.log 2>&1 || { tail -30 $OUT/ff.log; exit 1; }
tail -1 $OUT/ff.log
RTW_LIB=$LIB timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/parity.log 2>&1 || { tail -30 $OUT/parity.log; exit 1; }
tail -1 $OUT/parity.log
bash tools/ab_shard_r03.sh $1 3 '1:0 8:4' raytracing_in_a_weekend_rust_amd/_lib/librtw.so $LIB
