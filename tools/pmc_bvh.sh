# instruction-mix / wait counters of one render (separate --pmc passes, no tracing)
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONPATH=.
OUT=gpurun_out/pmc_${TAG:-bvh}; CMD=${CMD:-"bench.py --steps 1 --warmup 0 --cpu-baseline 0"}
mkdir -p $OUT
run() { timeout -k 10 300 rocprofv3 --pmc "$@" -d $OUT/p$N -o run --output-format csv -- python3 $CMD > $OUT/p$N.log 2>&1; N=$((N+1)); }
N=1
run SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES
run SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE
run SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_INT32 SQ_LDS_BANK_CONFLICT
python3 - $OUT <<'PY'
import csv, glob, sys, collections
for f in sorted(glob.glob(sys.argv[1] + "/p*/**/*counter_collection.csv", recursive=True)):
    d = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        if "rtw_" in r["Kernel_Name"]:
            d[r["Kernel_Name"][:60]][r["Counter_Name"]] += float(r["Counter_Value"])
    for k, v in d.items():
        print(k, {a: f"{b:.4g}" for a, b in v.items()})
PY
