set -o pipefail
mkdir -p gpurun_out/s4m
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused.py -x -q --timeout 120 --timeout-method thread > gpurun_out/s4m/fused_tests.log 2>&1 || { tail -30 gpurun_out/s4m/fused_tests.log; exit 1; }
tail -1 gpurun_out/s4m/fused_tests.log
timeout -k 10 120 python tools/kbench.py --ops fused --levels 0,1,2 --tag "auto" 2>/dev/null >> gpurun_out/s4m/kb.txt || exit 1
for f in "" "0,1" "0,1,2" "0,1"; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --fused-levels "$f" 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('fused=$f', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'])" >> gpurun_out/s4m/ab.txt || exit 1
done
cat gpurun_out/s4m/kb.txt | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['level'], d['tag'], d['us'])"
cat gpurun_out/s4m/ab.txt
