set -o pipefail
mkdir -p gpurun_out/g18; rm -f gpurun_out/g18/var.txt
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/ > gpurun_out/g18/tests.txt 2>&1 || { tail -30 gpurun_out/g18/tests.txt; exit 1; }
tail -2 gpurun_out/g18/tests.txt
for lv in 2 3; do timeout -k 10 200 python tools/variants.py --op corr --level $lv --knobs "rows_lanes8=0" >> gpurun_out/g18/var.txt 2>&1 || exit 1; done
for lv in 2 3; do timeout -k 10 100 python tools/rows_phases.py --level $lv >> gpurun_out/g18/var.txt 2>&1 || exit 1; done
