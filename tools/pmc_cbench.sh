#!/bin/bash
# PMC counters for corr kernels in tools/cbench (one rocprofv3 pass per counter group).
#   bash tools/pmc_cbench.sh <ONLY-filter> <kernel-regex> <outdir> [B C H W]
set -o pipefail
FILT=$1; REGEX=$2; OUT=$3; shift 3
SHAPE=${@:-8 32 96 112}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
run() { name=$1; shift; ONLY=$FILT WARM=20 timeout -k 10 120 rocprofv3 --pmc "$@" --kernel-include-regex "$REGEX" -d $OUT/$name -o run --output-format csv -- ./tools/cbench $SHAPE 20 > $OUT/$name.log 2>&1 || { echo "$name failed"; exit 1; }; }
run sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS
run sq2 SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_VMEM GRBM_GUI_ACTIVE SQ_WAIT_INST_LDS
run sq3 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MFMA_F32 SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM_WR SQ_ACTIVE_INST_VMEM SQ_INSTS_SMEM SQ_INSTS_VMEM_WR SQ_INSTS_LDS
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
