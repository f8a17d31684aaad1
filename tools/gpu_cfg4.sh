#!/bin/bash
# BASELINE config 4 bench line (B=16 448x1024 fp16) + rocprof kernel stats of it
set -o pipefail
OUT=gpurun_out/cfg4; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py --dtype fp16 --batch 16 --height 448 --width 1024 --steps 100 --warmup 10 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python bench.py --dtype fp16 --batch 16 --height 448 --width 1024 --steps 100 --warmup 10 --no-cpu-baseline > $OUT/bench_traced.json 2> $OUT/trace.err || exit 1
tail -c 1500 $OUT/bench.json
