#!/bin/bash
# Phase census of the l4 strip geometries under the measurement ablations built as
# tools/strip_bench_abl<mask> (-DPWC_STRIP_CENSUS -DPWC_STRIP_ABL=mask: 1 no stores, 2 no window
# reads after step 0, 4 no FMAs, 8 no f1 prefetch) -> $OUT
OUT=${OUT:-gpurun_out/strip_abl}
GEOS=${GEOS:-4 6}
ABLS=${ABLS:-1 2 4 8 14}
mkdir -p $OUT
for g in $GEOS; do
  for a in $ABLS; do
    PWC_DEBUG=strip_geo=$g timeout -k 10 60 tools/strip_bench_abl$a 300 > $OUT/abl${a}_$g.txt 2>&1 || { tail -3 $OUT/abl${a}_$g.txt; exit 1; }
    echo "abl=$a geo=$g $(tail -1 $OUT/abl${a}_$g.txt)"; tail -2 $OUT/abl${a}_$g.txt | head -1 | cut -c1-900
  done
done
