#!/bin/bash
# the strip correlation backward at small batches (B = 1, 2, 4) against the row-band
# kernel (knob bwd_strip=0; bwd_strip=2 forces the strip kernel at any grid), l2-l4 of 384x448, kbench --backward -> $OUT
set -o pipefail
OUT=${OUT:-gpurun_out/bwd_small}
mkdir -p $OUT
for B in 1 2 4; do
  for k in "bwd_strip=2" "bwd_strip=0"; do
    PWC_DEBUG=$k timeout -k 10 200 python tools/kbench.py --batch $B --levels 2,3,4 --ops none --backward > $OUT/b${B}_${k:-strip}.txt 2>&1 || { tail $OUT/b${B}_${k:-strip}.txt; exit 1; }
    echo "B=$B ${k:-strip}: $(grep -o '"level": [0-9], "op": "corr_bwd", "shape": [^]]*], "us": [0-9.]*' $OUT/b${B}_${k:-strip}.txt | sed 's/"shape": \[[^]]*\], //;s/"level": //;s/"op": "corr_bwd", //;s/"us": //' | tr '\n' ' ')"
  done
done
