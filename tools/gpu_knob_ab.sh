#!/bin/bash
# A/B of PWC_DEBUG knob settings ($KNOBS, space-separated; "-" = none) on tools/kbench.py $KARGS,
# alternating, $ROUNDS rounds -> $OUT
set -o pipefail
OUT=${OUT:-gpurun_out/knob_ab}
mkdir -p $OUT
for r in $(seq ${ROUNDS:-2}); do
  for k in $KNOBS; do
    [ "$k" = "-" ] && kk="" || kk="$k"
    PWC_DEBUG=$kk timeout -k 10 200 python tools/kbench.py $KARGS > $OUT/${k}_$r.txt 2>&1 || { tail $OUT/${k}_$r.txt; exit 1; }
    echo "$k $r: $(grep -o '"level": [0-9], "op": "[a-z_0-9]*", "shape": [^]]*], "us": [0-9.]*' $OUT/${k}_$r.txt | sed 's/"shape": \[[^]]*\], //;s/"level": //;s/"op": //;s/"us": //' | tr '\n' ' ')"
  done
done
