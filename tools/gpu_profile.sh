#!/bin/bash
# Round profile -> $OUT (default gpurun_out/prof): GPU suite under a kernel trace (+ kernel
# coverage), smoke, the default bench (live PMC, CPU baselines, Corr4 line, Net forward), its
# rocprofv3 kernel stats, the training step (+ kernel stats), config 4 (+ kernel stats), and
# the strip kernels' standalone timing / census.  Every GPU step under its own time limit.
set -o pipefail
OUT=${OUT:-gpurun_out/prof}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/tests_trace -o run --output-format csv -- python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/ --deselect tests/test_gpu_multirank.py::test_two_ranks_on_one_gpu_over_gloo > $OUT/gputests.txt 2>&1 || { tail -30 $OUT/gputests.txt; exit 1; }
grep -E 'passed|failed' $OUT/gputests.txt
# the two-rank rehearsal spawns its own ranks: outside the profiler
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_multirank.py > $OUT/gputests_multirank.txt 2>&1 || { tail -30 $OUT/gputests_multirank.txt; exit 1; }
tail -1 $OUT/gputests_multirank.txt
python tools/kernel_coverage.py $OUT/tests_trace/run_kernel_stats.csv > $OUT/coverage.txt || exit 1
head -1 $OUT/coverage.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.txt 2>&1 || { tail $OUT/smoke.txt; exit 1; }
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/bench_trace -o run --output-format csv -- python bench.py --no-cpu-baseline --no-pmc --no-net-forward --no-corr4 --grouped-mode off > $OUT/bench_traced.json 2> $OUT/bench_trace.err || { tail $OUT/bench_trace.err; exit 1; }
timeout -k 10 300 python tools/train_bench.py > $OUT/train.json 2> $OUT/train.err || { tail $OUT/train.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/train_trace -o run --output-format csv -- python tools/train_bench.py --grouped-mode off --no-kernels > $OUT/train_traced.json 2> $OUT/train_trace.err || { tail $OUT/train_trace.err; exit 1; }
timeout -k 10 300 python bench.py --dtype fp16 --batch 16 --height 448 --width 1024 --no-cpu-baseline --no-net-forward > $OUT/cfg4.json 2> $OUT/cfg4.err || { tail $OUT/cfg4.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/cfg4_trace -o run --output-format csv -- python bench.py --dtype fp16 --batch 16 --height 448 --width 1024 --no-cpu-baseline --no-pmc --no-net-forward --no-corr4 --grouped-mode off > $OUT/cfg4_traced.json 2> $OUT/cfg4_trace.err || { tail $OUT/cfg4_trace.err; exit 1; }
# (the strip census binary is a local measurement build; it does not travel with the tree)
if [ -x tools/strip_bench_census ]; then
  timeout -k 10 120 tools/strip_bench_census 300 > $OUT/strip_census.txt 2>&1 || { tail $OUT/strip_census.txt; exit 1; }
fi
echo done
