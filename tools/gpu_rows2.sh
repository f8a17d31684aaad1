set -o pipefail
mkdir -p gpurun_out/rows2; rm -f gpurun_out/rows2/kb.txt
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k corr_forward > gpurun_out/rows2/parity.log 2>&1 || { tail -30 gpurun_out/rows2/parity.log; exit 1; }
tail -1 gpurun_out/rows2/parity.log
PWC_ROWS=0 timeout -k 10 120 python tools/kbench.py --ops corr --levels 2,3,4 --tag off 2>/dev/null >> gpurun_out/rows2/kb.txt || exit 1
for c in "3,16" "2,16" "1,16" "3,8" "2,8" "1,8" "4,8"; do
  PWC_ROWS_CFG=$c timeout -k 10 120 python tools/kbench.py --ops corr --levels 2,3,4 --tag "rows$c" 2>/dev/null >> gpurun_out/rows2/kb.txt || exit 1
done
python3 -c "
import json
for l in open('gpurun_out/rows2/kb.txt'):
    d=json.loads(l); print(d['level'], d['op'], d['tag'], d['us'])"
