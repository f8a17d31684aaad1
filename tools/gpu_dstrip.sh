#!/bin/bash
# Standalone check + timing of the l4 displacement-diagonal strip (corr_dstrip.hip, strip_geo=20)
# against the whole-row strip (GeoF, strip_geo=10): tools/strip_bench, warm and cold -> $OUT
set -o pipefail
OUT=${OUT:-gpurun_out/dstrip}
mkdir -p $OUT
for g in ${GEOS:-20 10}; do
  PWC_DEBUG=strip_geo=$g timeout -k 10 60 tools/strip_bench 300 > $OUT/w_$g.txt 2>&1 || { cat $OUT/w_$g.txt; exit 1; }
  grep max_abs $OUT/w_$g.txt; tail -1 $OUT/w_$g.txt
  PWC_DEBUG=strip_geo=$g STRIP_SETS=24 timeout -k 10 60 tools/strip_bench 300 > $OUT/c_$g.txt 2>&1 || { cat $OUT/c_$g.txt; exit 1; }
  tail -1 $OUT/c_$g.txt
done
