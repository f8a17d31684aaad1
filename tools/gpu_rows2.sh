#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/rows2
timeout -k 10 300 python -u -m pytest tests/ -m gpu -x -q -k "corr or level or sintel or net or cat or fused" --timeout 120 --timeout-method thread > gpurun_out/rows2/pytest.log 2>&1 || { tail -30 gpurun_out/rows2/pytest.log; exit 1; }
tail -1 gpurun_out/rows2/pytest.log
OPS="corr:2 corr:3" KNOBS="rows=0" bash tools/gpu_variants.sh
for l in 0 1 2; do timeout -k 10 200 python tools/variants.py --op corr --level $l --dtype fp16 --batch 16 --height 448 --width 1024 --knobs "rows_r=1,rows_ck=32;rows_r=2,rows_ck=32;rows_r=1,rows_ck=48" 2>&1 | grep us; done
