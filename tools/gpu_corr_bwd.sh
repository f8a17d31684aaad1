#!/bin/bash
# corr_bwd: backward parity tests, then per-level times of the default path
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_train_step.py -k "backward or train or corr_back or autograd or cvl or Cost or cost" > gpurun_out/cbwd_tests.txt 2>&1 || { tail -30 gpurun_out/cbwd_tests.txt; exit 1; }
tail -1 gpurun_out/cbwd_tests.txt
for l in 4 3 2 1 0; do timeout -k 10 200 python tools/variants.py --op corr_bwd --level $l --knobs "$KNOBS" 2>&1 | grep us | cut -c1-150; done
