set -euo pipefail
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp PYTHONPATH=.
O=gpurun_out/pair4; mkdir -p $O
for v in 0 1; do
  RTW_AB=1 RTW_PAIR=$v timeout -k 10 300 python bench.py --shard-of 8:4 --cpu-baseline 0 --e2e 0 --steps 3 --warmup 1 > $O/bench_shard8_4_pair$v.json 2> $O/bench_shard8_4_pair$v.err
  RTW_AB=1 RTW_PAIR=$v timeout -k 10 300 python tools/diag_events.py 23 8 4 > $O/events_n8r4_pair$v.log 2>&1
  echo "pair=$v done"
done
for L in base cur; do for ROW in 308 455; do
  echo "== $L row $ROW" >> $O/chain.log
  CHAIN_ROW=$ROW RTW_LIB=$(realpath ab/$L/librtw.so) timeout -k 10 120 python -u tools/chain.py 2>&1 | grep "^\[" >> $O/chain.log
done; done
cat $O/chain.log
timeout -k 10 900 python -u tools/libab.py 6 ab/base/librtw.so ab/cur/librtw.so ab/lane/librtw.so > $O/libab.log 2>&1; tail -4 $O/libab.log
