#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/p2
timeout -k 10 300 python -u -m pytest tests/test_gpu_config4.py -x -q --timeout 120 --timeout-method thread > gpurun_out/p2/pytest.log 2>&1 || { tail -30 gpurun_out/p2/pytest.log; exit 1; }
tail -1 gpurun_out/p2/pytest.log
