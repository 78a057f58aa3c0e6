# instruction-cache and instruction-wait counters of one bench render (separate --pmc passes)
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONPATH=.
OUT=gpurun_out/pmc_${TAG:-icache}; CMD=${CMD:-"bench.py --steps 1 --warmup 0 --cpu-baseline 0"}
mkdir -p $OUT
run() { timeout -k 10 300 rocprofv3 --pmc "$@" -d $OUT/p$N -o run --output-format csv -- python3 $CMD > $OUT/p$N.log 2>&1; N=$((N+1)); }
N=1
run SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE
run SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU
run SQC_TC_INST_REQ SQC_TC_STALL SQC_ICACHE_BUSY_CYCLES SQ_ACTIVE_INST_ANY
python3 - $OUT <<'PY'
import csv, glob, sys, collections
for f in sorted(glob.glob(sys.argv[1] + "/p*/**/*counter_collection.csv", recursive=True)):
    d = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        if "rtw_render" in r["Kernel_Name"] or "finish" in r["Kernel_Name"]:
            d[r["Kernel_Name"][:60]][r["Counter_Name"]] += float(r["Counter_Value"])
    for k, v in d.items():
        print(k, {a: f"{b:.4g}" for a, b in v.items()})
PY
