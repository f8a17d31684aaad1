#!/bin/bash
# round-2 first GPU pass: parity tests, copy-floor probe, bench, rocprof kernel stats of bench
set -o pipefail
OUT=gpurun_out/r02a
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 120 ./tools/floor_probe > $OUT/floor.txt 2>&1 || exit 1
cat $OUT/floor.txt
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python bench.py --no-cpu-baseline > $OUT/bench_traced.json 2> $OUT/trace.err || { tail $OUT/trace.err; exit 1; }
echo done
