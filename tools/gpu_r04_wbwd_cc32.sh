# round 4: warp backward merged launch at l3 with 32 grad_x channels per tile workgroup (half the
# list builds; build/ab_cc32) vs 16 (tree): parity of the variant, then kbench --backward
set -o pipefail
mkdir -p gpurun_out
PWC_HOTPATH_LIB=build/ab_cc32/libpwc_hotpath.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "warp" > gpurun_out/cc32_tests.txt 2>&1 || { tail -20 gpurun_out/cc32_tests.txt; exit 1; }
tail -1 gpurun_out/cc32_tests.txt
for i in 1 2; do
  for v in cc32 tree; do
    if [ $v = cc32 ]; then export PWC_HOTPATH_LIB=build/ab_cc32/libpwc_hotpath.so; else unset PWC_HOTPATH_LIB; fi
    timeout -k 10 120 python tools/kbench.py --backward --ops warp --levels 2,3 > gpurun_out/cc32_k.log 2>&1 || { tail gpurun_out/cc32_k.log; exit 1; }
    echo "$v $(grep -o '"level": [0-9], "op": "warp_bwd".*"us": [0-9.]*' gpurun_out/cc32_k.log | sed 's/"shape.*"us"/us/' | tr '\n' ' ')"
  done
done
