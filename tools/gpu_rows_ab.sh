# bench A/B: default kernels vs corr_rows.hip at l3/l4 (PWC_ROWS=1), alternating, then the
# round profile of the default configuration
set -o pipefail
mkdir -p gpurun_out/rowsab
for v in def rows def rows; do
  if [ $v = rows ]; then export PWC_ROWS=1; else unset PWC_ROWS; fi
  timeout -k 10 200 python bench.py --no-cpu-baseline 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'])" >> gpurun_out/rowsab/ab.txt || exit 1
done
unset PWC_ROWS
cat gpurun_out/rowsab/ab.txt
bash tools/profile_round.sh ${1:-r01e}
