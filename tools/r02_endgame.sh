# GPU box: parity tests, N=1 A/B of builds, strong-scaling shard times (endgame + prepark rules)
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONPATH=.
OUT=gpurun_out/${TAG:-r02_endgame}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 600 python -u tools/libab.py 3 $LIBS > $OUT/ab.log 2>&1 || { tail -20 $OUT/ab.log; exit 1; }
tail -3 $OUT/ab.log
timeout -k 10 300 python tools/shard_time.py 1 2 4 8 > $OUT/shard_time.log 2>&1; grep "N=" $OUT/shard_time.log
timeout -k 10 120 python tools/diag_pix.py 23 8 0 > $OUT/diag_n8r0.log 2>&1; sed -n 1,2p $OUT/diag_n8r0.log; grep -E "timeline|last|heaviest" $OUT/diag_n8r0.log
