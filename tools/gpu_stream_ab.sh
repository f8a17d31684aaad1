#!/bin/bash
# l4 stream-kernel ablations / configurations (PWC_DEBUG knobs), kbench l4 corr each
set -o pipefail
OUT=gpurun_out/stream_ab
mkdir -p $OUT; : > $OUT/ab.txt
for v in "stream_abl=6" "stream_abl=14" "stream_abl=22" "stream_abl=46" "stream_abl=54" "stream_abl=38" "stream_abl=0"; do
  PWC_DEBUG=$v timeout -k 10 120 python tools/kbench.py --levels 4 --ops corr --iters 60 2>/dev/null | grep corr_fwd | sed "s/^/$v /" >> $OUT/ab.txt || exit 1
done
cat $OUT/ab.txt
