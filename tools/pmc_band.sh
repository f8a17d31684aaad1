set -o pipefail
mkdir -p gpurun_out/s4k
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export PWC_BAND_CFG=3,1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY -d gpurun_out/s4k/p1 -o p1 --output-format csv --kernel-include-regex "band|corr_fwd_small|sm_reduce|warp_fwd" -- python tools/kbench.py --ops corr,fused --levels 0 --iters 5 > gpurun_out/s4k/p1.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_SMEM SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM_RD SQ_INSTS_BRANCH SQ_ACTIVE_INST_LDS -d gpurun_out/s4k/p2 -o p2 --output-format csv --kernel-include-regex "band|corr_fwd_small|sm_reduce|warp_fwd" -- python tools/kbench.py --ops corr,fused --levels 0 --iters 5 > gpurun_out/s4k/p2.log 2>&1 || exit 1
python3 tools/pmc_agg.py gpurun_out/s4k/p1 --delete > gpurun_out/s4k/p1.json && python3 tools/pmc_agg.py gpurun_out/s4k/p2 --delete > gpurun_out/s4k/p2.json && cat gpurun_out/s4k/p1.json gpurun_out/s4k/p2.json
