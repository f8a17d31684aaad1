# round 4: matrix-core strip C = 96 geometry (config-4 l2): parity tests, kbench A/B against the
# previous build (build/ab_old: row-band kernel at l2), then the config-4 bench
set -o pipefail
mkdir -p gpurun_out/m96
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_coverage.py tests/test_gpu_config4.py tests/test_gpu_parity.py > gpurun_out/m96/t.log 2>&1; rc=$?; tail -2 gpurun_out/m96/t.log; [ $rc -eq 0 ] || exit $rc
K="--batch 16 --height 448 --width 1024 --dtype fp16 --levels 2,3,4 --ops corr"
for i in 1 2; do
  for L in build/ab_old pwc-net_pytorch_amd/pwcnet_amd/lib; do
    PWC_HOTPATH_LIB=$L/libpwc_hotpath.so timeout -k 10 120 python tools/kbench.py $K > gpurun_out/m96/k.log 2>&1 || exit 1
    echo "$L $(grep corr_fwd gpurun_out/m96/k.log | python -c 'import sys,json;print([(json.loads(l)["level"], json.loads(l)["us"]) for l in sys.stdin])')"
  done
done
timeout -k 10 300 python bench.py --dtype fp16 --batch 16 --height 448 --width 1024 --no-cpu-baseline --no-net-forward --no-corr4 > gpurun_out/m96/cfg4.json 2> gpurun_out/m96/cfg4.err || { tail gpurun_out/m96/cfg4.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/m96/cfg4.json').read().strip().splitlines()[-1]);print('cfg4', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['frac'], d['roofline'].get('traffic'))"
