# corr_bwd: parity tests, then per-level times and the l4/l3 census
set -o pipefail
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_train_step.py -k "backward or train or corr_back or autograd or cvl or Cost or cost" > gpurun_out/cbwd_tests.txt 2>&1 || { tail -30 gpurun_out/cbwd_tests.txt; exit 1; }
tail -1 gpurun_out/cbwd_tests.txt
for l in 4 3 2 1 0; do timeout -k 10 200 python tools/variants.py --op corr_bwd --level $l --knobs "" || exit 1; done 2>&1 | grep -v amdgpu.ids | cut -c1-120
for l in 4 3; do timeout -k 10 100 python tools/bwd_phases.py --level $l || exit 1; done 2>&1 | grep -v amdgpu.ids
