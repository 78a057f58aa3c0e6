set -euo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONPATH=.
OUT=gpurun_out/early; mkdir -p $OUT
for rep in 1 2 3; do
  for L in kp tir early; do
    echo "== $L rep $rep" >> $OUT/st.log
    RTW_LIB=$(realpath ab/$L/librtw.so) timeout -k 10 200 python -u tools/shard_time.py 4 8 2>&1 | grep "^N=" >> $OUT/st.log
  done
done
RTW_LIB=$(realpath ab/early/librtw.so) timeout -k 10 300 python -u tools/knob_sweep.py 8:4,8:0,8:1,4:0 ';RTW_EARLY_K=2;RTW_EARLY_K=3;RTW_EARLY_K=6;RTW_EARLY_X=16;RTW_EARLY_X=28;RTW_EARLY_K=4294967295' > $OUT/sweep.log 2>&1
cat $OUT/st.log; cat $OUT/sweep.log
