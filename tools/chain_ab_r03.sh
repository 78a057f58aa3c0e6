# Round-3: drain-chain latency of one image row, A/B of library builds (alternating).
# Usage: bash tools/chain_ab_r03.sh TAG ROWS LIB...
set -euo pipefail
cd "$GRAFT_REPO_ROOT"; export PYTHONPATH=. TMPDIR=/tmp
OUT=gpurun_out/$1; ROWS=$2; shift 2; mkdir -p $OUT
for rep in 1 2; do for row in $ROWS; do for lib in "$@"; do
  echo "row $row lib $lib" >> $OUT/chain.log
  CHAIN_ROW=$row RTW_LIB=$lib timeout -k 10 120 python -u tools/chain.py RTW_BUDGET_X=0.01 2>&1 | grep -v amdgpu >> $OUT/chain.log
done; done; done
cat $OUT/chain.log
