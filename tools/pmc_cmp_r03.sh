# PMC comparison of library builds (main kernel counters per dispatch, 1e9 units).
# Usage: LIBS='name:path name:path' bash tools/pmc_cmp_r03.sh
set -e
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp PYTHONPATH=.
mkdir -p gpurun_out/r03_pb
P="insts=SQ_INSTS_VALU,SQ_INSTS_SALU,SQ_INSTS_LDS,SQ_INSTS_VALU_TRANS_F64,SQ_INSTS_VALU_FMA_F64,SQ_INSTS_VALU_MUL_F64,SQ_INSTS_VALU_ADD_F64,SQ_INSTS_SMEM cyc=SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_VALU,SQ_ACTIVE_INST_ANY,SQ_THREAD_CYCLES_VALU lds=SQ_LDS_BANK_CONFLICT,SQ_LDS_IDX_ACTIVE,SQ_WAIT_INST_LDS,SQ_ACTIVE_INST_LDS,SQ_INSTS_VMEM,SQ_ACTIVE_INST_VMEM"
for L in ${LIBS:-main:raytracing_in_a_weekend_rust_amd/_lib/librtw.so}; do
  n=${L%%:*}; f=${L#*:}
  RTW_LIB=$f timeout -k 10 240 python -u tools/pmc_diag.py $P > gpurun_out/r03_pb/pmc_$n.json 2> gpurun_out/r03_pb/pmc_$n.err
done
LIBS="$LIBS" python - <<'PY'
import json
import os
for n in [x.split(':')[0] for x in os.environ.get('LIBS','main:').split()]:
    d=json.load(open(f'gpurun_out/r03_pb/pmc_{n}.json'))
    r={}
    for p,v in d.items():
        for k,c in v.items():
            if 'persist' in k: r.update(c)
    print(n, json.dumps({k:round(v/1e9,3) for k,v in sorted(r.items())}))
PY
