# round 4: matrix-core strip, eight compute waves and one accumulated tile per block: parity
# tests, kbench A/B against the four-wave build (build/ab_old) and the eight-wave two-tile build
# (build/ab_mid), census-build ablations
set -o pipefail
mkdir -p gpurun_out/m8
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_coverage.py tests/test_gpu_config4.py "tests/test_gpu_parity.py::test_correlation_properties_sintel_fp16" > gpurun_out/m8/t.log 2>&1; rc=$?; tail -2 gpurun_out/m8/t.log; [ $rc -eq 0 ] || exit $rc
K="--batch 16 --height 448 --width 1024 --dtype fp16 --levels 3,4 --ops corr"
for i in 1 2; do
  for L in build/ab_old build/ab_mid pwc-net_pytorch_amd/pwcnet_amd/lib; do
    PWC_HOTPATH_LIB=$L/libpwc_hotpath.so timeout -k 10 120 python tools/kbench.py $K > gpurun_out/m8/k.log 2>&1 || exit 1
    echo "$L $(grep corr_fwd gpurun_out/m8/k.log | python -c 'import sys,json;print([(json.loads(l)["level"], json.loads(l)["us"]) for l in sys.stdin])')"
  done
done
for a in 0 1 2 6; do
  PWC_HOTPATH_LIB=build/census/libpwc_hotpath.so PWC_DEBUG=ms_abl=$a timeout -k 10 60 python tools/kbench.py $K > gpurun_out/m8/abl_$a.log 2>&1 || exit 1
  echo "ms_abl=$a $(grep corr_fwd gpurun_out/m8/abl_$a.log | python -c 'import sys,json;print([(json.loads(l)["level"], json.loads(l)["us"]) for l in sys.stdin])')"
done
