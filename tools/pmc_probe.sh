#!/bin/bash
# PMC counters for one kernel of tools/kbench.py, one rocprofv3 pass per counter group.
#   bash tools/pmc_probe.sh <kernel-regex> <levels> <outdir> [extra env assignments...]
set -o pipefail
REGEX=${1:-corr_fwd_ring}; LEVELS=${2:-4}; OUT=${3:-gpurun_out/pmc}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
run() { name=$1; shift; timeout -k 10 120 rocprofv3 --pmc "$@" --kernel-include-regex "$REGEX" -d $OUT/$name -o run --output-format csv -- python tools/kbench.py --levels $LEVELS --iters 10 > $OUT/$name.log 2>&1; echo "$name rc=$?"; }
run sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS
run sq2 SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_VMEM GRBM_GUI_ACTIVE SQ_WAIT_INST_LDS
run sq3 SQ_INSTS_VALU_FMA_F32 SQ_LEVEL_WAVES SQ_INST_LEVEL_LDS SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_SCA
run ta1 TA_BUSY_avr TA_BUFFER_READ_LDS_WAVEFRONTS_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum
run tcc1 FETCH_SIZE
run tcc2 WRITE_SIZE
for f in $OUT/*/run_counter_collection.csv; do python3 - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(list)
for r in rows:
    agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in agg.items():
    print(f"{k:40s} n={len(v):4d} mean={sum(v)/len(v):.1f}")
PY
done
