#!/bin/bash
# Phase census (tools/strip_bench_census) and a no-store ablation (tools/strip_bench_nostore:
# every output store discarded by the range check) of the l4 strip geometries in $GEOS -> $OUT
OUT=${OUT:-gpurun_out/strip_census}
GEOS=${GEOS:-4 5 6 7}
mkdir -p $OUT
for g in $GEOS; do
  PWC_DEBUG=strip_geo=$g timeout -k 10 60 tools/strip_bench_census 300 > $OUT/census_$g.txt 2>&1 || { cat $OUT/census_$g.txt; exit 1; }
  tail -2 $OUT/census_$g.txt
  PWC_DEBUG=strip_geo=$g timeout -k 10 60 tools/strip_bench_nostore 300 > $OUT/nostore_$g.txt 2>&1 || { cat $OUT/nostore_$g.txt; exit 1; }
  tail -1 $OUT/nostore_$g.txt
done
