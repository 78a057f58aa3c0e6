# GPU box: A/B of the two-lane walk split (RTW_PAIR) -- parity with the split forced on
# every render, then the strong split (N=8 ranks) and N=1 with and without it.
set -euo pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp PYTHONPATH=.
O=gpurun_out/${TAG:-pair}; mkdir -p $O
if [ "${PARITY:-1}" = 1 ]; then
  RTW_AB=1 RTW_PAIR=2 timeout -k 10 500 python -u -m pytest tests/test_gpu_fullframe.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "not config5" > $O/parity_pair2.log 2>&1 || { tail -30 $O/parity_pair2.log; exit 1; }
  tail -1 $O/parity_pair2.log; grep -m2 "RTW_PAIR" $O/parity_pair2.log || true
fi
for i in $(seq 1 ${REPS:-2}); do
  RTW_AB=1 RTW_PAIR=1 timeout -k 10 300 python -u tools/shard_time.py ${NS:-1 8} > $O/st_pair1_$i.log 2>&1
  grep "^N=" $O/st_pair1_$i.log | sed 's/^/pair /'; grep -m1 "RTW_PAIR" $O/st_pair1_$i.log || true
  RTW_AB=1 RTW_PAIR=2 timeout -k 10 300 python -u tools/shard_time.py ${NS:-1 8} > $O/st_pair2_$i.log 2>&1
  grep "^N=" $O/st_pair2_$i.log | sed 's/^/pair2 /'; grep -m1 "RTW_PAIR" $O/st_pair2_$i.log || true
  timeout -k 10 300 python -u tools/shard_time.py ${NS:-1 8} > $O/st_base_$i.log 2>&1
  grep "^N=" $O/st_base_$i.log | sed 's/^/base /'
done
