set -o pipefail
mkdir -p gpurun_out/g14
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/ > gpurun_out/g14/tests.txt 2>&1 || { tail -30 gpurun_out/g14/tests.txt; exit 1; }
tail -2 gpurun_out/g14/tests.txt
timeout -k 10 300 python tools/train_bench.py > gpurun_out/g14/train.json 2> gpurun_out/g14/train.err
