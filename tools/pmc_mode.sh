# SQ_INSTS_VALU / SALU / wave cycles of one bench render under the knob settings in $KNOBS
# (e.g. parking off: how many VALU instructions the drain groups cost)
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONPATH=.
OUT=gpurun_out/pmc_mode_${TAG:-x}
mkdir -p $OUT
env $KNOBS timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_INSTS_LDS -d $OUT/p -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --cpu-baseline 0 > $OUT/p.log 2>&1
python3 tools/pmc_insts.py $OUT p
