# budget x accel sweep under rocprofv3 kernel trace: per-kernel (phase 1 / phase 2) times
set -euo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONPATH=.
OUT=${SWEEP_OUT:-gpurun_out/sweep}
mkdir -p $OUT
for cfg in ${CFGS:-"2:6:64:768" "2:10:64:768" "2:6:64:1024" "2:0:64:768"}; do
  IFS=: read a b c pb rx hv cg <<< "$cfg"
  pb=${pb:-768}; rx=${rx:-16}; hv=${hv:-1}; cg=${cg:-16}
  RTW_COOPG=$cg RTW_RATE_X=$rx RTW_HEAVY=$hv RTW_PBLOCK=$pb RTW_COOP=$c RTW_ACCEL=$a RTW_BUDGET_X=$b timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/t_${a}_${b}_${pb}_${rx}_${hv}_${cg} -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --cpu-baseline 0 > $OUT/b_${a}_${b}_${pb}_${rx}_${hv}_${cg}.json 2> $OUT/b_${a}_${b}_${pb}_${rx}_${hv}_${cg}.err
  echo "== accel $a budget $b coop $c pblock $pb rate $rx heavy $hv coopg $cg"
  python3 -c "import json;d=json.load(open('$OUT/b_${a}_${b}_${pb}_${rx}_${hv}_${cg}.json'));print(d['ms_per_step'], d['stats'])"
  grep -h "rtw_" $OUT/t_${a}_${b}_${pb}_${rx}_${hv}_${cg}/*kernel_stats.csv | cut -d, -f1-4
done
