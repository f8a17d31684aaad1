#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/cbwd
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fused.py tests/test_net_harness.py -x -q -k "backward or autograd or grad or net" --timeout 120 --timeout-method thread > gpurun_out/cbwd/pytest.log 2>&1 || { tail -30 gpurun_out/cbwd/pytest.log; exit 1; }
tail -1 gpurun_out/cbwd/pytest.log
timeout -k 10 200 python tools/kbench.py --iters 40 --ops corr --backward 2>&1 | grep corr_bwd
timeout -k 10 200 python tools/train_bench.py
