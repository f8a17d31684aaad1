#!/bin/bash
# Census + ablations of the l4 diagonal strip (tools/strip_bench_dcensus, strip_bench_dabl<mask>:
# 1 no stores, 2 no FMAs, 4 no window reads) -> $OUT
set -o pipefail
OUT=${OUT:-gpurun_out/dstrip_abl}
mkdir -p $OUT
timeout -k 10 60 tools/strip_bench_dcensus 300 > $OUT/census.txt 2>&1 || { cat $OUT/census.txt; exit 1; }
grep census $OUT/census.txt; tail -1 $OUT/census.txt
for a in ${ABLS:-1 2 4 6}; do
  timeout -k 10 60 tools/strip_bench_dabl$a 300 > $OUT/abl$a.txt 2>&1 || { cat $OUT/abl$a.txt; exit 1; }
  echo "abl $a: $(tail -1 $OUT/abl$a.txt)"
done
for v in ${VARIANTS:-dn2 dn4}; do
  timeout -k 10 60 tools/strip_bench_$v 300 > $OUT/$v.txt 2>&1 || { cat $OUT/$v.txt; exit 1; }
  echo "$v: $(grep max_abs $OUT/$v.txt) $(tail -1 $OUT/$v.txt)"
done
if [ -x tools/strip_bench_dcensus2 ]; then
  timeout -k 10 60 tools/strip_bench_dcensus2 300 > $OUT/census2.txt 2>&1 || { cat $OUT/census2.txt; exit 1; }
  grep census $OUT/census2.txt
fi
