# Round-3: parity tests, then every rank of the N=1,2,4,8 strong splits on one GPU.
# Usage: bash tools/verify_r03.sh TAG
set -euo pipefail
cd "$GRAFT_REPO_ROOT"; export PYTHONPATH=. TMPDIR=/tmp
OUT=gpurun_out/$1; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python -u tools/shard_time.py 1 2 4 8 > $OUT/shard_time.log 2>&1
grep -v amdgpu $OUT/shard_time.log
