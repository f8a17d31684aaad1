#!/bin/bash
# Round-3 profile -> gpurun_out/prof_r03: GPU tests under a kernel trace (kernel coverage),
# smoke, the bench (live PMC + CPU baselines), its rocprofv3 kernel stats, the training step
# (JSON + kernel stats) and config 4.
set -o pipefail
OUT=${OUT:-gpurun_out/prof_r03}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/tests_trace -o run --output-format csv -- python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/ > $OUT/gputests.txt 2>&1 || { tail -30 $OUT/gputests.txt; exit 1; }
tail -2 $OUT/gputests.txt
python tools/kernel_coverage.py $OUT/tests_trace/run_kernel_stats.csv > $OUT/coverage.txt || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.txt 2>&1 || { tail $OUT/smoke.txt; exit 1; }
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/bench_trace -o run --output-format csv -- python bench.py --no-cpu-baseline --no-pmc --grouped-mode off > $OUT/bench_traced.json 2> $OUT/bench_trace.err || { tail $OUT/bench_trace.err; exit 1; }
timeout -k 10 300 python tools/train_bench.py > $OUT/train.json 2> $OUT/train.err || { tail $OUT/train.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/train_trace -o run --output-format csv -- python tools/train_bench.py --grouped-mode off --no-kernels > $OUT/train_traced.json 2> $OUT/train_trace.err || { tail $OUT/train_trace.err; exit 1; }
timeout -k 10 300 python bench.py --dtype fp16 --batch 16 --height 448 --width 1024 --no-cpu-baseline > $OUT/cfg4.json 2> $OUT/cfg4.err || { tail $OUT/cfg4.err; exit 1; }
echo done
