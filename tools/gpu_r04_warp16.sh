# round 4: fp16 warp with one 8-byte load per sample-row pair: warp / config-4 tests, kbench A/B
# of the fp16 warps (config-4 l2..l4) against the previous build (build/ab_old)
set -o pipefail
mkdir -p gpurun_out/w16
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_coverage.py tests/test_gpu_config4.py tests/test_gpu_parity.py > gpurun_out/w16/t.log 2>&1; rc=$?; tail -2 gpurun_out/w16/t.log; [ $rc -eq 0 ] || exit $rc
K="--batch 16 --height 448 --width 1024 --dtype fp16 --levels 1,2,3,4 --ops warp"
for i in 1 2; do
  for L in build/ab_old pwc-net_pytorch_amd/pwcnet_amd/lib; do
    PWC_HOTPATH_LIB=$L/libpwc_hotpath.so timeout -k 10 120 python tools/kbench.py $K > gpurun_out/w16/k.log 2>&1 || exit 1
    echo "$L $(grep warp_fwd gpurun_out/w16/k.log | python -c 'import sys,json;print([(json.loads(l)["level"], json.loads(l)["us"]) for l in sys.stdin])')"
  done
done
