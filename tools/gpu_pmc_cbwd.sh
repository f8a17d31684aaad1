#!/bin/bash
# SQ counters of the l4 correlation backward (two passes)
set -o pipefail
cd $GRAFT_REPO_ROOT
export OP=corr_bwd LEVEL=${LEVEL:-4} KRE=corr_bwd
CTRS="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT" bash tools/gpu_pmc_op.sh > gpurun_out/pmc_cbwd_a.txt 2>&1 && cat gpurun_out/pmc_cbwd_a.txt &&
mv gpurun_out/pmc_corr_bwd_l$LEVEL gpurun_out/pmc_corr_bwd_l${LEVEL}_a &&
CTRS="SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAIT_ANY GRBM_GUI_ACTIVE" bash tools/gpu_pmc_op.sh > gpurun_out/pmc_cbwd_b.txt 2>&1 && cat gpurun_out/pmc_cbwd_b.txt
