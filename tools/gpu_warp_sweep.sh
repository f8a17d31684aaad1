#!/bin/bash
# warp forward variants (knob warp_cfg) at l2..l4, random N(0,2^2) flows and zero flow
set -o pipefail
OUT=gpurun_out/warp_sweep
mkdir -p $OUT; : > $OUT/w.txt
for v in 0 1 2 3 5 6 7 8 9; do
  PWC_DEBUG=warp_cfg=$v timeout -k 10 100 python tools/kbench.py --ops warp --levels 2,3,4 --iters 40 --tag cfg$v 2>/dev/null | grep warp_fwd >> $OUT/w.txt || exit 1
done
timeout -k 10 100 python tools/kbench.py --ops warp --levels 2,3,4 --iters 40 --flow-scale 0 --tag zero 2>/dev/null | grep warp_fwd >> $OUT/w.txt || exit 1
cat $OUT/w.txt
