set -o pipefail
mkdir -p gpurun_out/full
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/full/tests.log 2>&1 || { tail -60 gpurun_out/full/tests.log; exit 1; }
tail -2 gpurun_out/full/tests.log
