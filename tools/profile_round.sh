#!/bin/bash
# Round profile: bench JSON, per-level kernel times (kbench), rocprofv3 kernel-trace stats of
# the same bench command, and the PMC passes (FETCH_SIZE / WRITE_SIZE, one counter per pass)
# for the l4 correlation kernel.  Writes gpurun_out/prof_<tag>.
# (Round 1 recipe: its PMC passes name corr_fwd_ring, the l4 kernel of rounds 1-2, removed in round 3.)
set -o pipefail
TAG=${1:-r01}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --cpu-seconds 10 > $OUT/bench.json 2> $OUT/bench.err || exit 1
timeout -k 10 200 python tools/kbench.py --iters 60 --ops corr,warp,fused,upwarp --backward > $OUT/kbench.txt 2>&1 || exit 1
timeout -k 10 200 python tools/train_bench.py > $OUT/train.json 2> $OUT/train.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python bench.py --steps 200 --warmup 20 --no-cpu-baseline > $OUT/bench_traced.json 2> $OUT/trace.err || exit 1
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $ctr --kernel-include-regex corr_fwd_ring -d $OUT/pmc_$ctr -o run --output-format csv -- python tools/kbench.py --levels 4 --iters 20 > $OUT/pmc_$ctr.log 2>&1 || exit 1
done
echo done
