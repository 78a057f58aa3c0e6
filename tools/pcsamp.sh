# PC sampling (host trap) of one bench step: per-instruction hotspots of the render kernel
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONPATH=.
OUT=gpurun_out/pcs
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time --pc-sampling-interval ${PCS_INTERVAL:-100} -d $OUT -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --cpu-baseline 0 > $OUT/log.txt 2>&1 || { tail -20 $OUT/log.txt; exit 1; }
ls -la $OUT $OUT/* | head -30
