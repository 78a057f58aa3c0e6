# dry-cursor parking threshold x hot-wave priority: kernel time and completion timeline
set -euo pipefail
cd "$GRAFT_REPO_ROOT"; export PYTHONPATH=.
for hp in ${HOTPRIO:-0}; do for t in ${TAILS:-768}; do
  RTW_HOTPRIO=$hp RTW_TAIL=$t timeout -k 10 200 python tools/diag_pix.py 23 > gpurun_out/diag_t${t}_h$hp.log 2>&1
  echo "== tail $t hotprio $hp"; grep -E "kernel|timeline" gpurun_out/diag_t${t}_h$hp.log | cut -c1-300
done; done
