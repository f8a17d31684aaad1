#!/bin/bash
# PMC passes of ONE kernel (regex KRE) over any command, each pass a run of its own under
# `timeout -s KILL 60` (rocprofv3 does not split counters over passes):
#   sq   - instruction mix and wave states (8 SQ counters)
#   lds  - LDS array cycles, bank conflicts, LDS issue stalls (7 SQ + GRBM_GUI_ACTIVE)
#   tcc  - L2 hits / misses (all requests of the kernel)
#   fetch, write - FETCH_SIZE / WRITE_SIZE (HBM-side bytes; gfx950: FETCH_SIZE x 2 for 16-B
#          streaming reads, MI355X_MICROARCH.md "HBM")
# Means per launch are printed by tools/pmc_agg.py.
#   usage: KRE=corr_fwd_strip OUT=gpurun_out/pmc_x bash tools/gpu_pmc_kernel.sh python tools/kbench.py ...
set -o pipefail
OUT=${OUT:-gpurun_out/pmc}
PASSES=${PASSES:-sq lds fetch write}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
declare -A CTR
CTR[sq]="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD"
CTR[lds]="SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE"
CTR[tcc]="TCC_HIT_sum TCC_MISS_sum"
CTR[fetch]="FETCH_SIZE"
CTR[write]="WRITE_SIZE"
for p in $PASSES; do
  timeout -s KILL 60 rocprofv3 --pmc ${CTR[$p]} --kernel-include-regex "$KRE" -d $OUT/$p -o run \
    --output-format csv -- "$@" > $OUT/$p.log 2>&1 || { tail -5 $OUT/$p.log; exit 1; }
done
python tools/pmc_agg.py $OUT
