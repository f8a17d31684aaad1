#!/bin/bash
# kernel trace + counters of the l4 warp backward (gx lists + flow kernels)
set -o pipefail
cd $GRAFT_REPO_ROOT
export OP=warp_bwd LEVEL=${LEVEL:-4} KRE=warp_bwd
bash tools/gpu_trace_op.sh > gpurun_out/wbwd_trace.txt 2>&1 && cat gpurun_out/wbwd_trace.txt &&
CTRS="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" bash tools/gpu_pmc_op.sh > gpurun_out/pmc_wbwd_a.txt 2>&1 && cat gpurun_out/pmc_wbwd_a.txt &&
mv gpurun_out/pmc_warp_bwd_l$LEVEL gpurun_out/pmc_warp_bwd_l${LEVEL}_a &&
CTRS="TA_TA_BUSY_sum TA_FLAT_READ_WAVEFRONTS_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum FETCH_SIZE GRBM_GUI_ACTIVE" bash tools/gpu_pmc_op.sh > gpurun_out/pmc_wbwd_b.txt 2>&1 && cat gpurun_out/pmc_wbwd_b.txt
