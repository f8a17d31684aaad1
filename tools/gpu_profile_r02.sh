#!/bin/bash
# Round profile: PMC HBM bytes of the l4 correlation (FETCH_SIZE, WRITE_SIZE: one counter per
# pass), the training step of the hot path (JSON + rocprofv3 kernel stats), per-level kbench
# incl. backward.  -> gpurun_out/prof_r02
set -o pipefail
OUT=gpurun_out/prof_r02
mkdir -p $OUT
export TMPDIR=/tmp
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 90 rocprofv3 --pmc $ctr --kernel-include-regex corr_fwd_stream -d $OUT/pmc_$ctr -o run --output-format csv -- python tools/kbench.py --levels 4 --ops corr --iters 20 > $OUT/pmc_$ctr.log 2>&1 || { tail $OUT/pmc_$ctr.log; exit 1; }
done
python tools/pmc_summary.py $OUT/pmc_FETCH_SIZE/run_counter_collection.csv $OUT/pmc_WRITE_SIZE/run_counter_collection.csv $OUT/l4corr_pmc.json corr_fwd_stream || exit 1
timeout -k 10 200 python tools/train_bench.py > $OUT/train.json 2> $OUT/train.err || { tail $OUT/train.err; exit 1; }
cat $OUT/train.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/train_trace -o run --output-format csv -- python tools/train_bench.py > $OUT/train_traced.json 2> $OUT/train_trace.err || { tail $OUT/train_trace.err; exit 1; }
timeout -k 10 300 python tools/kbench.py --iters 40 --ops corr,warp,fused,upwarp --backward > $OUT/kbench.txt 2>&1 || { tail $OUT/kbench.txt; exit 1; }
echo done
