set -o pipefail
mkdir -p gpurun_out/g19
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/ > gpurun_out/g19/tests.txt 2>&1 || { tail -40 gpurun_out/g19/tests.txt; exit 1; }
tail -2 gpurun_out/g19/tests.txt
timeout -k 10 300 python bench.py --no-cpu-baseline --no-pmc --dtype fp16 --batch 16 --height 448 --width 1024 --steps 100 > gpurun_out/g19/cfg4.json 2> gpurun_out/g19/cfg4.err
