# round 4: the matrix-core fp16 strip kernel (corr_mstrip16.hip, C = 32 and C = 64 geometries):
# parity tests, then kbench A/B at config-4 l4 and l3 against the channel-pair stream kernel
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_coverage.py tests/test_gpu_config4.py "tests/test_gpu_parity.py::test_correlation_properties_sintel_fp16" > gpurun_out/m16.log 2>&1; rc=$?; tail -25 gpurun_out/m16.log; [ $rc -eq 0 ] || exit $rc
for k in mstrip16=1 mstrip16=0 mstrip16=1 mstrip16=0; do
  PWC_DEBUG=$k timeout -k 10 120 python tools/kbench.py --batch 16 --height 448 --width 1024 --dtype fp16 --levels 3,4 --ops corr > gpurun_out/km16.log 2>&1 || exit 1; echo "$k"; grep corr_fwd gpurun_out/km16.log
done
