set -o pipefail
mkdir -p gpurun_out/ab2
for v in ring pt ring pt; do
  if [ $v = pt ]; then export PWC_PT_L4=1; else unset PWC_PT_L4; fi
  timeout -k 10 200 python bench.py --no-cpu-baseline 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'])" >> gpurun_out/ab2/ab.txt || exit 1
done
