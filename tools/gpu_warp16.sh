#!/bin/bash
# fp16 warp variants at config-4 levels (warp_cfg knob)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/var
for lv in 4 3 2; do
  timeout -k 10 200 python tools/variants.py --op warp --level $lv --batch 16 --height 448 --width 1024 --dtype fp16 --knobs "warp_cfg=8;warp_cfg=6;warp_cfg=9;warp_cfg=5;warp_cfg=4;warp_cfg=2" > gpurun_out/var/warp16_l$lv.txt 2>&1 || { tail -3 gpurun_out/var/warp16_l$lv.txt; exit 1; }
  grep '^{' gpurun_out/var/warp16_l$lv.txt | cut -c1-130
done
