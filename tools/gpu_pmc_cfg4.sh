#!/bin/bash
# SQ counters of the config-4 l4 correlation (fp16, B=16, 112x256x32)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
OUT=gpurun_out/pmc_cfg4; mkdir -p $OUT
for pass in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT" "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAIT_ANY SQ_INST_CYCLES_VMEM_WR SQ_INSTS_VALU_DOT"; do
  tag=$(echo $pass | cut -c1-12 | tr ' ' _)
  timeout -s KILL 120 rocprofv3 --pmc $pass --kernel-include-regex corr_fwd_stream -d $OUT/$tag -o run --output-format csv -- python tools/variants.py --op corr --level 4 --batch 16 --height 448 --width 1024 --dtype fp16 --iters 5 > $OUT/log_$tag.txt 2>&1 || { tail $OUT/log_$tag.txt; exit 1; }
done
python - <<PY
import csv, glob, collections
acc = collections.defaultdict(list)
for f in glob.glob("$OUT/**/run_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        acc[(r["Kernel_Name"][:50], r["Counter_Name"])].append(float(r["Counter_Value"]))
for k, v in sorted(acc.items()):
    print(k, round(sum(v)/len(v)))
PY
