#!/bin/bash
# Round profile TAG (default r02e) -> gpurun_out/prof_TAG: default bench (CPU baselines, live PMC traffic),
# graph-all comparison, rocprofv3 kernel stats of the bench, committed-PMC summary of the l4
# correlation, per-level kbench incl. backward, training step (+ kernel stats), config 4.
set -o pipefail
OUT=$GRAFT_REPO_ROOT/gpurun_out/prof_${TAG:-r02e}
mkdir -p $OUT
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
timeout -k 10 400 python $R/bench.py --cpu-seconds 10 > $OUT/bench_full.json 2> $OUT/bench_full.err || { tail $OUT/bench_full.err; exit 1; }
echo bench done
timeout -k 10 300 python $R/bench.py --no-cpu-baseline --no-pmc --timing graph-all > $OUT/bench_graph_all.json 2> $OUT/bench_graph_all.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python $R/bench.py --no-cpu-baseline --no-pmc > $OUT/bench_traced.json 2> $OUT/trace.err || { tail $OUT/trace.err; exit 1; }
echo trace done
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-include-regex corr_fwd_stream -d $OUT/pmc_$ctr -o run --output-format csv -- python $R/tools/kbench.py --levels 4 --ops corr --iters 20 > $OUT/pmc_$ctr.log 2>&1 || { tail $OUT/pmc_$ctr.log; exit 1; }
done
python $R/tools/pmc_summary.py $(ls $OUT/pmc_FETCH_SIZE/*/run_counter_collection.csv $OUT/pmc_FETCH_SIZE/run_counter_collection.csv 2>/dev/null | head -1) $(ls $OUT/pmc_WRITE_SIZE/*/run_counter_collection.csv $OUT/pmc_WRITE_SIZE/run_counter_collection.csv 2>/dev/null | head -1) $OUT/l4corr_pmc.json corr_fwd_stream > /dev/null || exit 1
echo pmc done
timeout -k 10 300 python $R/tools/kbench.py --iters 40 --ops corr,warp,fused,upwarp --backward > $OUT/kbench.txt 2>&1 || { tail $OUT/kbench.txt; exit 1; }
timeout -k 10 200 python $R/tools/train_bench.py > $OUT/train.json 2> $OUT/train.err || { tail $OUT/train.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/train_trace -o run --output-format csv -- python $R/tools/train_bench.py > $OUT/train_traced.json 2> $OUT/train_trace.err || exit 1
echo train done
timeout -k 10 300 python $R/bench.py --dtype fp16 --batch 16 --height 448 --width 1024 --no-cpu-baseline > $OUT/cfg4_bench.json 2> $OUT/cfg4.err || { tail $OUT/cfg4.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/cfg4_trace -o run --output-format csv -- python $R/bench.py --dtype fp16 --batch 16 --height 448 --width 1024 --no-cpu-baseline --no-pmc > $OUT/cfg4_traced.json 2> $OUT/cfg4_trace.err || exit 1
echo all done
