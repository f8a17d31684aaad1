#!/bin/bash
# A/B of the l4 strip geometries standalone (tools/strip_bench, no torch): warm (default sets),
# cold (STRIP_SETS=24) and the census build, for each PWC_DEBUG strip_geo in $GEOS -> $OUT
GEOS=${GEOS:-5 4}
OUT=${OUT:-gpurun_out/strip_ab}
set -o pipefail
mkdir -p $OUT
for geo in $GEOS; do
  PWC_DEBUG=strip_geo=$geo timeout -k 10 120 tools/strip_bench 300 > $OUT/sb_$geo.txt 2>&1 || { cat $OUT/sb_$geo.txt; exit 1; }
  tail -2 $OUT/sb_$geo.txt
  PWC_DEBUG=strip_geo=$geo STRIP_SETS=24 timeout -k 10 120 tools/strip_bench 300 > $OUT/sb_cold_$geo.txt 2>&1 || { cat $OUT/sb_cold_$geo.txt; exit 1; }
  tail -1 $OUT/sb_cold_$geo.txt
  PWC_DEBUG=strip_geo=$geo timeout -k 10 120 tools/strip_bench_census 300 > $OUT/census_$geo.txt 2>&1 || { cat $OUT/census_$geo.txt; exit 1; }
  tail -2 $OUT/census_$geo.txt
done
