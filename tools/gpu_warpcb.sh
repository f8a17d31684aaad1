#!/bin/bash
set -o pipefail
K="warp_cfg=5;warp_cfg=10;warp_cfg=11;warp_cfg=7"
for l in 2 3 4; do timeout -k 10 200 python tools/variants.py --op warp --level $l --knobs "$K" 2>&1 | grep us; done
for l in 2 3 4; do timeout -k 10 200 python tools/variants.py --op warp --level $l --dtype fp16 --batch 16 --height 448 --width 1024 --knobs "$K" 2>&1 | grep us; done
