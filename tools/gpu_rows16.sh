#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/rows16
timeout -k 10 300 python -u -m pytest tests/test_gpu_config4.py -x -q --timeout 120 --timeout-method thread > gpurun_out/rows16/pytest.log 2>&1 || { tail -30 gpurun_out/rows16/pytest.log; exit 1; }
tail -1 gpurun_out/rows16/pytest.log
for l in 0 1 2; do
timeout -k 10 200 python tools/variants.py --op corr --level $l --dtype fp16 --batch 16 --height 448 --width 1024 --knobs "rows=0" 2>&1 | grep us
done
