# Round-3 diagnosis on the GPU box: per-rank times of the strong split (N=1,2,4,8
# on one GPU), per-pixel timelines of the slowest ranks, LDS/VALU counter passes
# of the full frame, and the build-stamped PMC file for profiles/.
# Usage: bash tools/strong_r03.sh TAG
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONPATH=.
OUT=gpurun_out/$1
mkdir -p $OUT
timeout -k 10 300 python -u tools/shard_time.py 1 2 4 8 > $OUT/shard_time.log 2>&1
cat $OUT/shard_time.log
timeout -k 10 120 python -u tools/diag_pix.py 23 8 4 > $OUT/diag_n8_r4.log 2>&1
timeout -k 10 120 python -u tools/diag_pix.py 23 4 0 > $OUT/diag_n4_r0.log 2>&1
timeout -k 10 300 python -u tools/pmc_diag.py \
  lds=SQ_LDS_IDX_ACTIVE,SQ_LDS_BANK_CONFLICT,SQ_WAIT_INST_LDS,SQ_ACTIVE_INST_LDS,SQ_WAIT_INST_ANY,SQ_WAVE_CYCLES,SQ_ACTIVE_INST_ANY,SQ_BUSY_CYCLES,GRBM_GUI_ACTIVE \
  valu=SQ_THREAD_CYCLES_VALU,SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_SCA,SQ_ACTIVE_INST_MISC,SQ_ACTIVE_INST_VMEM,SQ_INSTS_BRANCH,SQ_INSTS_SMEM,SQ_INST_CYCLES_SALU,GRBM_GUI_ACTIVE \
  > $OUT/pmc_diag.json 2> $OUT/pmc_diag.err
timeout -k 10 400 python bench.py --cpu-baseline 0 --e2e 0 --pmc-out $OUT/r03_pmc.json > $OUT/bench.json 2> $OUT/bench.err
cat $OUT/bench.json
