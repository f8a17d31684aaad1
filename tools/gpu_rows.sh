# corr_rows.hip (row-band correlation) on the GPU: parity with PWC_ROWS=1, then per-level
# timings against the default kernels over its (R, CK) configurations (tools/kbench.py)
set -o pipefail
mkdir -p gpurun_out/rows
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k corr_forward"
timeout -k 10 300 $T > gpurun_out/rows/parity_default.log 2>&1 || { tail -30 gpurun_out/rows/parity_default.log; exit 1; }
PWC_ROWS=1 timeout -k 10 300 $T > gpurun_out/rows/parity_rows.log 2>&1 || { tail -30 gpurun_out/rows/parity_rows.log; exit 1; }
timeout -k 10 120 python tools/kbench.py --ops corr --levels 2,3,4 --tag default 2>/dev/null >> gpurun_out/rows/kb.txt || exit 1
for c in "3,16" "3,8" "2,16" "2,8" "1,16" "4,16"; do
  PWC_ROWS=1 PWC_ROWS_CFG=$c timeout -k 10 120 python tools/kbench.py --ops corr --levels 2,3,4 --tag "rows$c" 2>/dev/null >> gpurun_out/rows/kb.txt || exit 1
done
tail -2 gpurun_out/rows/parity_default.log gpurun_out/rows/parity_rows.log
python3 -c "
import json
for l in open('gpurun_out/rows/kb.txt'):
    d=json.loads(l); print(d['level'], d['op'], d['tag'], d['us'])"
