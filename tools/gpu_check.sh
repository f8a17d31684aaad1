# full GPU test suite, then bench A/B of a kernel switch: gpu_check.sh <ENVVAR> <value-for-B>
set -o pipefail
mkdir -p gpurun_out/chk
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/chk/tests.log 2>&1 || { tail -40 gpurun_out/chk/tests.log; exit 1; }
tail -3 gpurun_out/chk/tests.log
if [ -n "$1" ]; then
  rm -f gpurun_out/chk/ab.txt
  for v in A B A B; do
    if [ $v = B ]; then export $1=$2; else unset $1; fi
    timeout -k 10 200 python bench.py --no-cpu-baseline 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'])" >> gpurun_out/chk/ab.txt || exit 1
  done
  cat gpurun_out/chk/ab.txt
fi
