#!/bin/bash
# PMC counters of one variants.py op: OP, LEVEL, CTRS (one pass), KRE (kernel regex)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/pmc_${OP}_l${LEVEL}; mkdir -p $OUT
timeout -s KILL 120 rocprofv3 --pmc $CTRS --kernel-include-regex "$KRE" -d $OUT -o run --output-format csv -- python tools/variants.py --op $OP --level $LEVEL --iters 5 > $OUT/log.txt 2>&1 || { tail $OUT/log.txt; exit 1; }
python - <<PY
import csv, glob, collections
f = glob.glob("$OUT/**/run_counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    acc[(r["Kernel_Name"][:40], r["Counter_Name"])].append(float(r["Counter_Value"]))
for k, v in sorted(acc.items()):
    print(k, round(sum(v)/len(v)))
PY
