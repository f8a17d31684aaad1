#!/bin/bash
# warp forward: timing against flow scale (gather coherence) + counters at l4
set -o pipefail
cd $GRAFT_REPO_ROOT
export OP=warp LEVEL=${LEVEL:-4} KRE=warp_fwd
for fs in 0 0.5 2 4; do
  timeout -k 10 120 python tools/variants.py --op warp --level $LEVEL --iters 300 --flow-scale $fs --knobs "warp_cfg=3;warp_cfg=8" || exit 1
done
CTRS="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" bash tools/gpu_pmc_op.sh > gpurun_out/pmc_wfwd_a.txt 2>&1 && cat gpurun_out/pmc_wfwd_a.txt &&
mv gpurun_out/pmc_warp_l$LEVEL gpurun_out/pmc_warp_l${LEVEL}_a &&
CTRS="TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum FETCH_SIZE GRBM_GUI_ACTIVE" bash tools/gpu_pmc_op.sh > gpurun_out/pmc_wfwd_b.txt 2>&1 && cat gpurun_out/pmc_wfwd_b.txt &&
mv gpurun_out/pmc_warp_l$LEVEL gpurun_out/pmc_warp_l${LEVEL}_b &&
CTRS="TD_TD_BUSY_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum WRITE_SIZE" bash tools/gpu_pmc_op.sh > gpurun_out/pmc_wfwd_c.txt 2>&1 && cat gpurun_out/pmc_wfwd_c.txt
