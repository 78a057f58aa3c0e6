# Instruction-cache counters of one frame (the persistent kernel is 78 KB of code;
# the CU pair's instruction cache is smaller). Usage: bash tools/r05_icache.sh TAG [LIB]
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONPATH=.
OUT=gpurun_out/$1
mkdir -p $OUT
LIB=${2:-}
env ${LIB:+RTW_LIB=$(realpath $LIB)} timeout -k 10 300 python tools/pmc_diag.py icache=SQC_ICACHE_REQ,SQC_ICACHE_HITS,SQC_ICACHE_MISSES,SQC_ICACHE_MISSES_DUPLICATE,SQ_IFETCH,SQ_WAVE_CYCLES,SQC_ICACHE_INPUT_VALID_READYB,SQ_BUSY_CYCLES > $OUT/pmc_icache.json 2> $OUT/pmc_icache.err
python3 -c "
import json;d=json.load(open('$OUT/pmc_icache.json'))['icache']
for k,v in d.items():
    if v.get('SQ_WAVE_CYCLES',0)>1e6: print(k, {c:('%.4g'%x) for c,x in v.items()}, 'hit %.4f' % (v['SQC_ICACHE_HITS']/max(v['SQC_ICACHE_REQ'],1)))
"
