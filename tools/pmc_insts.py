#!/usr/bin/env python3
"""Per-launch instruction counts of the persistent render kernel from a rocprofv3
--pmc pass (SQ_INSTS_* count wave-level instructions). The bulk of the launch is
limited by VALU issue and latency: on gfx950 a wave64 f32/int VALU instruction
occupies the SIMD for 2 cycles, an f64 one for 4 (bench.py valu_issue).
Usage: pmc_insts.py OUTDIR [PASS [KERNEL]]  (expects OUTDIR/PASS, default pmc_insts;
KERNEL defaults to the parity kernel, rtw_fast_render for the f32 fast mode)."""
import csv
import glob
import json
import os
import sys

KERNEL = "rtw_render_persist"


def main():
    out = sys.argv[1]
    sub = sys.argv[2] if len(sys.argv) > 2 else "pmc_insts"
    kernel = sys.argv[3] if len(sys.argv) > 3 else KERNEL
    acc, launches = {}, {}
    for f in glob.glob(os.path.join(out, sub, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if kernel in row["Kernel_Name"]:
                    n = row["Counter_Name"]
                    acc[n] = acc.get(n, 0.0) + float(row["Counter_Value"])
                    launches.setdefault(n, set()).add(row.get("Dispatch_Id", row.get("Correlation_Id", "")))
    res = {"workload": "complex_1200x675_s23_d50", "kernel": kernel}
    for n, v in sorted(acc.items()):
        res[n.lower() + "_per_launch"] = v / max(1, len(launches[n]))
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
