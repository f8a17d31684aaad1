#!/bin/bash
# Same-box A/B of library builds in the bench step: bench.py (no CPU baseline / PMC / Net /
# Corr4 / grouped mode) alternating the in-tree library and each PWC_HOTPATH_LIB in $LIBS,
# $ROUNDS times; one line per run: value, ms_per_step, l4 event us.  Extra bench args: $ARGS
LIBS=${LIBS:-}
ROUNDS=${ROUNDS:-2}
for r in $(seq $ROUNDS); do
  for lib in tree $LIBS; do
    if [ $lib = tree ]; then L=""; else L=$lib; fi
    PWC_HOTPATH_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline --no-pmc --no-net-forward --no-corr4 --grouped-mode off $ARGS 2> gpurun_out/.ab.err > gpurun_out/.ab.json || { tail -5 gpurun_out/.ab.err; exit 1; }
    python -c "import json; d=json.loads(open('gpurun_out/.ab.json').read().strip().splitlines()[-1]); print('$lib', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'])"
  done
done
