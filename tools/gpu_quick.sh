#!/bin/bash
# GPU test suite under a kernel trace + coverage report, then the config-4 bench -> $OUT
set -o pipefail
OUT=${OUT:-gpurun_out/quick}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/tests_trace -o run --output-format csv -- python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/ > $OUT/gputests.txt 2>&1 || { grep -v rocprofv3 $OUT/gputests.txt | tail -30; exit 1; }
grep "passed\|failed" $OUT/gputests.txt | tail -1
python tools/kernel_coverage.py $OUT/tests_trace/run_kernel_stats.csv > $OUT/coverage.txt || exit 1
head -1 $OUT/coverage.txt
timeout -k 10 300 python bench.py --dtype fp16 --batch 16 --height 448 --width 1024 --no-cpu-baseline > $OUT/cfg4.json 2> $OUT/cfg4.err || { tail $OUT/cfg4.err; exit 1; }
python -c "import json; c=json.load(open('$OUT/cfg4.json')); print('cfg4', c['ms_per_step'], c['grouped']['ms_per_step'] if 'grouped' in c else '')"
