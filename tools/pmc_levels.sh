# SQ instruction / cycle counters of the unfused kernels at l2..l4 (kbench), aggregated per kernel
set -o pipefail
mkdir -p gpurun_out/pmcl
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
R='corr_fwd_stream|corr_fwd_rows|corr_fwd_pt|warp_fwd|warp_corr_band'
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VMEM_WR -d gpurun_out/pmcl/p1 -o p1 --output-format csv --kernel-include-regex "$R" -- python tools/kbench.py --ops corr,warp,fused --levels 0,1,2,3,4 --iters 5 > gpurun_out/pmcl/p1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_INSTS_VALU_FMA_F32 SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM -d gpurun_out/pmcl/p2 -o p2 --output-format csv --kernel-include-regex "$R" -- python tools/kbench.py --ops corr,warp,fused --levels 0,1,2,3,4 --iters 5 > gpurun_out/pmcl/p2.log 2>&1 || exit 1
python3 tools/pmc_agg.py gpurun_out/pmcl/p1 --delete > gpurun_out/pmcl/p1.json && python3 tools/pmc_agg.py gpurun_out/pmcl/p2 --delete > gpurun_out/pmcl/p2.json
