#!/bin/bash
# kernel-variant sweep: OPS="op:level ..." KNOBS="k1;k2" -> gpurun_out/var/<op>_l<level>.txt
set -o pipefail
mkdir -p gpurun_out/var
for ol in ${OPS:-corr:4}; do
  op=${ol%%:*}; lv=${ol##*:}
  timeout -k 10 200 python tools/variants.py --op $op --level $lv --knobs "${KNOBS}" > gpurun_out/var/${op}_l${lv}.txt 2>&1 || { tail -5 gpurun_out/var/${op}_l${lv}.txt; exit 1; }
  grep -v amdgpu.ids gpurun_out/var/${op}_l${lv}.txt | cut -c1-160
done
