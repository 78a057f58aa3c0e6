set -euo pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp PYTHONPATH=.
OUT=gpurun_out/$1; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VALU_TRANS_F64 -d $OUT/pmc_insts -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --cpu-baseline 0 > $OUT/pmc_insts.log 2>&1
python3 tools/pmc_insts.py $OUT > $OUT/pmc_insts.json
cat $OUT/pmc_insts.json
