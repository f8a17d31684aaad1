#!/bin/bash
# Round-4 check: GPU suite under a kernel trace (+ kernel coverage), then the default bench.
set -o pipefail
OUT=${OUT:-gpurun_out/r04t}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 700 rocprofv3 --kernel-trace --stats -d $OUT/tests_trace -o run --output-format csv -- python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/ > $OUT/gputests.txt 2>&1 || { tail -30 $OUT/gputests.txt; exit 1; }
tail -2 $OUT/gputests.txt
python tools/kernel_coverage.py $OUT/tests_trace/run_kernel_stats.csv > $OUT/coverage.txt || exit 1
head -1 $OUT/coverage.txt
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
cat $OUT/bench.json
