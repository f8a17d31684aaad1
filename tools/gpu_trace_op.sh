#!/bin/bash
# per-kernel durations of one variants.py op (rocprofv3 kernel trace): OP, LEVEL, KNOBS
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/trace_${OP}_l${LEVEL}_fs${FS:-2}; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- python tools/variants.py --op $OP --level $LEVEL --knobs "${KNOBS}" --iters 20 --flow-scale ${FS:-2} > $OUT/log.txt 2>&1 || { tail $OUT/log.txt; exit 1; }
python - <<PY
import csv, glob
f = glob.glob("$OUT/**/run_kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:12]:
    print(r["Calls"], round(float(r["AverageNs"])/1000, 2), r["Name"][:100])
PY
