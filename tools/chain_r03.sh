set -euo pipefail
cd "$GRAFT_REPO_ROOT"; export PYTHONPATH=. TMPDIR=/tmp; mkdir -p gpurun_out/chain1
CHAIN_ROW=308 timeout -k 10 120 python -u tools/chain.py - RTW_BUDGET_X=0.01 > gpurun_out/chain1/row308.log 2>&1
CHAIN_ROW=468 timeout -k 10 120 python -u tools/chain.py - RTW_BUDGET_X=0.01 > gpurun_out/chain1/row468.log 2>&1
CHAIN_ROW=308 RTW_BUDGET_X=10 RTW_LIB=raytracing_in_a_weekend_rust_amd/_lib/librtw_stamps.so timeout -k 10 120 python -u tools/chain_stamps.py > gpurun_out/chain1/stamps308.log 2>&1
CHAIN_ROW=468 RTW_BUDGET_X=10 RTW_LIB=raytracing_in_a_weekend_rust_amd/_lib/librtw_stamps.so timeout -k 10 120 python -u tools/chain_stamps.py > gpurun_out/chain1/stamps468.log 2>&1
