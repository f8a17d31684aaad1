#!/bin/bash
# A/B of a measurement library build (tools/build_variant.sh -> $VLIB) against the in-tree
# library: tools/kbench.py $KARGS, alternating, $ROUNDS rounds -> $OUT
set -o pipefail
OUT=${OUT:-gpurun_out/lib_ab}
mkdir -p $OUT
for r in $(seq ${ROUNDS:-2}); do
  for v in base var; do
    if [ $v = var ]; then export PWC_HOTPATH_LIB=$VLIB; else unset PWC_HOTPATH_LIB; fi
    timeout -k 10 200 python tools/kbench.py $KARGS > $OUT/${v}_$r.txt 2>&1 || { tail $OUT/${v}_$r.txt; exit 1; }
    echo "$v $r: $(grep -o '"level": [0-9], "op": "[a-z_0-9]*", "shape": [^]]*], "us": [0-9.]*' $OUT/${v}_$r.txt | sed 's/"shape": \[[^]]*\], //;s/"level": //;s/"op": //;s/"us": //' | tr '\n' ' ')"
  done
done
