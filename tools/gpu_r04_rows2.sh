# round 4: row-band correlation with two chunks' loads in flight (plans whose registers fit):
# parity tests, kbench A/B (fp32 config 2 and fp16 config 4 levels) against build/ab_old
set -o pipefail
mkdir -p gpurun_out/r2
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/ > gpurun_out/r2/t.log 2>&1; rc=$?; tail -2 gpurun_out/r2/t.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  for L in build/ab_old pwc-net_pytorch_amd/pwcnet_amd/lib; do
    PWC_HOTPATH_LIB=$L/libpwc_hotpath.so timeout -k 10 120 python tools/kbench.py --levels 2,3 --ops corr > gpurun_out/r2/k.log 2>&1 || exit 1
    PWC_HOTPATH_LIB=$L/libpwc_hotpath.so timeout -k 10 120 python tools/kbench.py --batch 16 --height 448 --width 1024 --dtype fp16 --levels 1 --ops corr >> gpurun_out/r2/k.log 2>&1 || exit 1
    echo "$L $(grep corr_fwd gpurun_out/r2/k.log | python -c 'import sys,json;print([(json.loads(l)["level"], json.loads(l)["shape"][0], json.loads(l)["us"]) for l in sys.stdin])')"
  done
done
