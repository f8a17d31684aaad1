set -o pipefail
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_config4.py tests/test_gpu_coverage.py "tests/test_gpu_parity.py::test_correlation_properties_sintel_fp16" "tests/test_gpu_parity.py::test_level2_full_size_corr9_b8" > gpurun_out/t16.log 2>&1; rc=$?; tail -15 gpurun_out/t16.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python tools/kbench.py --batch 16 --height 448 --width 1024 --dtype fp16 --levels 4 --ops corr > gpurun_out/k16.log 2>&1; tail -3 gpurun_out/k16.log
PWC_DEBUG=strip16=0 timeout -k 10 120 python tools/kbench.py --batch 16 --height 448 --width 1024 --dtype fp16 --levels 4 --ops corr > gpurun_out/k16b.log 2>&1; tail -3 gpurun_out/k16b.log
