# instruction-mix counters + bench with new stats
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONPATH=.
OUT=gpurun_out/mix
mkdir -p $OUT
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --cpu-baseline 0 > $OUT/bench.json 2> $OUT/bench.err
cat $OUT/bench.json
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 -d $OUT/p1 -o run --output-format csv -- python bench.py --steps 1 --warmup 0 --cpu-baseline 0 > $OUT/p1.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU -d $OUT/p2 -o run --output-format csv -- python bench.py --steps 1 --warmup 0 --cpu-baseline 0 > $OUT/p2.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_INST_CYCLES_VALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_SMEM -d $OUT/p3 -o run --output-format csv -- python bench.py --steps 1 --warmup 0 --cpu-baseline 0 > $OUT/p3.log 2>&1
echo done
