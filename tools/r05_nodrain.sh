set -euo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONPATH=.
OUT=gpurun_out/r05_nodrain
mkdir -p $OUT
timeout -k 10 300 python tools/pmc_diag.py insts=SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_ACTIVE_INST_VALU,SQ_THREAD_CYCLES_VALU > $OUT/pmc_default.json 2> $OUT/pmc_default.err
env RTW_AB=1 RTW_BUDGET_X=0 RTW_RATE_X=0 RTW_HEAVY=0 RTW_TAIL=4294967295 RTW_JOIN=0 timeout -k 10 300 python tools/pmc_diag.py insts=SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_WAVE_CYCLES,SQ_WAIT_ANY,SQ_ACTIVE_INST_VALU,SQ_THREAD_CYCLES_VALU > $OUT/pmc_nodrain.json 2> $OUT/pmc_nodrain.err
env RTW_AB=1 RTW_BUDGET_X=0 RTW_RATE_X=0 RTW_HEAVY=0 RTW_TAIL=4294967295 RTW_JOIN=0 timeout -k 10 300 python bench.py --steps 2 --warmup 1 --cpu-baseline 0 --pmc 0 --e2e 0 > $OUT/bench_nodrain.json 2> $OUT/bench_nodrain.err
for f in default nodrain; do python3 -c "import json;d=json.load(open('$OUT/pmc_$f.json'))['insts']['rtw_render_persist'];print('$f', 'valu %.3fe9 salu %.3fe9 wave_cycles %.3fe12 wait %.4f lanes %.4f' % (d['SQ_INSTS_VALU']/1e9, d['SQ_INSTS_SALU']/1e9, d['SQ_WAVE_CYCLES']/1e12, d['SQ_WAIT_ANY']/d['SQ_WAVE_CYCLES'], d['SQ_THREAD_CYCLES_VALU']/(64*d['SQ_ACTIVE_INST_VALU'])))"; done
python3 -c "import json;d=json.load(open('$OUT/bench_nodrain.json'));print('nodrain', d['ms_per_step'], d['stats']['parked_pixels'], d['stats']['segments'])"
