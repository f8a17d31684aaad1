#!/bin/bash
# bench JSON + rocprof kernel stats of the same bench command -> gpurun_out/$1
set -o pipefail
OUT=gpurun_out/${1:-bp}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python bench.py ${BENCH_ARGS:---no-cpu-baseline} > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/bench.json')); print(d['value'], d['ms_per_step'], d['checks']['replay'], d['roofline']['avg_launch_us'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python bench.py --no-cpu-baseline > $OUT/bench_traced.json 2> $OUT/trace.err || { tail $OUT/trace.err; exit 1; }
python - "$OUT" <<'PY'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1] + '/trace/run_kernel_stats.csv')))[:7]:
    print(r['Name'][:70], r['Calls'], r['AverageNs'])
PY
