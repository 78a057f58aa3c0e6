# instruction counts of one bench render (one --pmc pass): the bulk is VALU-issue bound,
# so SQ_INSTS_VALU is the number to drive down
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONPATH=.
OUT=gpurun_out/pmc_${TAG:-insts}
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 -d $OUT/p -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --cpu-baseline 0 > $OUT/p.log 2>&1
python3 - $OUT <<'PY'
import csv, glob, sys, collections
for f in sorted(glob.glob(sys.argv[1] + "/p/**/*counter_collection.csv", recursive=True)):
    d = collections.defaultdict(float)
    for r in csv.DictReader(open(f)):
        if "rtw_render_persist" in r["Kernel_Name"]:
            d[r["Counter_Name"]] += float(r["Counter_Value"])
    seg = 1282991212 / 64
    print({a: f"{b:.4g} ({b / seg:.0f}/wave-seg)" for a, b in sorted(d.items())})
PY
