#!/bin/bash
set -o pipefail
OUT=gpurun_out/sbench
mkdir -p $OUT; : > $OUT/s.txt
for v in "stream_abl=0" "stream_abl=4" "stream_abl=7" "stream_abl=6"; do
  echo -n "$v " >> $OUT/s.txt
  PWC_DEBUG=$v timeout -k 10 60 ./tools/sbench 100 >> $OUT/s.txt 2>&1 || { cat $OUT/s.txt; exit 1; }
done
cat $OUT/s.txt
