#!/bin/bash
# Config-4 A/B of a measurement library ($VLIB) against the in-tree one: bench.py config 4 line
# (alternating, $ROUNDS rounds) and, per library, the PMC write / fetch passes of the matrix-core
# strip kernels -> $OUT
set -o pipefail
OUT=${OUT:-gpurun_out/cfg4_ab}
mkdir -p $OUT
ARGS="--dtype fp16 --batch 16 --height 448 --width 1024 --no-cpu-baseline --no-net-forward --no-corr4 --grouped-mode off --no-pmc"
for r in $(seq ${ROUNDS:-2}); do
  for v in base var; do
    if [ $v = var ]; then export PWC_HOTPATH_LIB=$VLIB; else unset PWC_HOTPATH_LIB; fi
    timeout -k 10 200 python bench.py $ARGS --steps 100 --warmup 100 > $OUT/${v}_$r.json 2> $OUT/${v}_$r.err || { tail $OUT/${v}_$r.err; exit 1; }
    echo "$v $r: $(python -c "import json;d=json.load(open('$OUT/${v}_$r.json'));print(d['value'], d['ms_per_step'], d.get('roofline',{}).get('achieved'))")"
  done
done
for v in base var; do
  if [ $v = var ]; then export PWC_HOTPATH_LIB=$VLIB; else unset PWC_HOTPATH_LIB; fi
  KRE=mstrip16 PASSES="fetch write" OUT=$OUT/pmc_$v bash tools/gpu_pmc_kernel.sh python bench.py $ARGS --steps 20 --warmup 20 || exit 1
done
