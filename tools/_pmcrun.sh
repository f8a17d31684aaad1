set -o pipefail
bash tools/pmc_cbench.sh parA_abl6 corr_fwd_par gpurun_out/pmc_parA6 > gpurun_out/pmc_parA6.txt 2>&1 || exit 1
bash tools/pmc_cbench.sh ringN_abl6 corr_fwd_ring gpurun_out/pmc_ringN6 > gpurun_out/pmc_ringN6.txt 2>&1 || exit 1
bash tools/pmc_cbench.sh parA corr_fwd_par gpurun_out/pmc_parA0 > gpurun_out/pmc_parA0.txt 2>&1 || exit 1
echo ok
