set -o pipefail
mkdir -p gpurun_out/g15
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/ > gpurun_out/g15/tests.txt 2>&1 || { tail -30 gpurun_out/g15/tests.txt; exit 1; }
tail -2 gpurun_out/g15/tests.txt
timeout -k 10 300 python bench.py --no-cpu-baseline --no-pmc > gpurun_out/g15/bench.json 2> gpurun_out/g15/bench.err
