# round 4: correlation backward with paired gO loads (lane pairs q = 0/1 swap halves) and the
# conflict-chosen LDS pitch -- parity tests, then kbench --backward l0..l4 against HEAD's build
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_coverage.py tests/test_train_step.py -k "bwd or backward or train or grad" > gpurun_out/bwdp_tests.txt 2>&1 || { tail -30 gpurun_out/bwdp_tests.txt; exit 1; }
tail -2 gpurun_out/bwdp_tests.txt
for i in 1 2; do
  PWC_HOTPATH_LIB=build/ab_old/libpwc_hotpath.so timeout -k 10 120 python tools/kbench.py --backward --ops corr > gpurun_out/bwdp_a.log 2>&1 || { tail gpurun_out/bwdp_a.log; exit 1; }
  echo "old:  $(grep corr_bwd gpurun_out/bwdp_a.log | tr '\n' ' ')"
  timeout -k 10 120 python tools/kbench.py --backward --ops corr > gpurun_out/bwdp_b.log 2>&1 || { tail gpurun_out/bwdp_b.log; exit 1; }
  echo "tree: $(grep corr_bwd gpurun_out/bwdp_b.log | tr '\n' ' ')"
done
