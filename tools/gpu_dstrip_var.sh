#!/bin/bash
# Timing of tools/strip_bench_<variant> builds of the l4 diagonal strip (+ GeoF for reference,
# + the census build when present) -> $OUT
set -o pipefail
OUT=${OUT:-gpurun_out/dstrip_var}
mkdir -p $OUT
PWC_DEBUG=strip_geo=10 timeout -k 10 60 tools/strip_bench 300 > $OUT/geof.txt 2>&1 || { cat $OUT/geof.txt; exit 1; }
echo "geof: $(tail -1 $OUT/geof.txt)"
for v in ${VARIANTS:-dv1 dv2 dv3 dv4}; do
  timeout -k 10 60 tools/strip_bench_$v 300 > $OUT/$v.txt 2>&1 || { cat $OUT/$v.txt; exit 1; }
  echo "$v: $(grep -o '"n_over_1e-5": [0-9]*' $OUT/$v.txt) $(tail -1 $OUT/$v.txt)"
done
if [ -x tools/strip_bench_dcensus ]; then
  timeout -k 10 60 tools/strip_bench_dcensus 300 > $OUT/census.txt 2>&1 || { cat $OUT/census.txt; exit 1; }
  grep census $OUT/census.txt
fi
