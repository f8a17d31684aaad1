#!/bin/bash
# Standalone timing of the l4 strip geometries compiled into tools/strip_bench (PWC_DEBUG
# strip_geo = 4..9), warm (default rotation) and cold (STRIP_SETS=24) -> $OUT
OUT=${OUT:-gpurun_out/strip_geos}
GEOS=${GEOS:-4 5 6 7 8 9}
mkdir -p $OUT
for g in $GEOS; do
  PWC_DEBUG=strip_geo=$g timeout -k 10 60 tools/strip_bench 300 > $OUT/w_$g.txt 2>&1 || { cat $OUT/w_$g.txt; exit 1; }
  tail -1 $OUT/w_$g.txt; grep max_abs $OUT/w_$g.txt
  PWC_DEBUG=strip_geo=$g STRIP_SETS=24 timeout -k 10 60 tools/strip_bench 300 > $OUT/c_$g.txt 2>&1 || { cat $OUT/c_$g.txt; exit 1; }
  tail -1 $OUT/c_$g.txt
done
