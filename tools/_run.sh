set -o pipefail
mkdir -p gpurun_out/st
L=pwc-net_pytorch_amd/pwcnet_amd/lib
for v in base v1 v2 base v2 v1; do
  if [ $v = base ]; then unset PWC_HOTPATH_LIB; else export PWC_HOTPATH_LIB=$PWD/$L/$v/libpwc_hotpath.so; fi
  timeout -k 10 200 python bench.py --no-cpu-baseline 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'])" >> gpurun_out/st/ab.txt || exit 1
done
export PWC_HOTPATH_LIB=$PWD/$L/v2/libpwc_hotpath.so
timeout -k 10 200 python tools/kbench.py --iters 60 > gpurun_out/st/kbench_v2.txt 2>&1 || exit 1
timeout -k 10 300 python -m pytest tests -m gpu -x -q > gpurun_out/st/pytest_v2.txt 2>&1 || exit 1
