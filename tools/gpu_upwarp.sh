set -o pipefail
mkdir -p gpurun_out/upw
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/upw/tests.log 2>&1 || { tail -40 gpurun_out/upw/tests.log; exit 1; }
tail -2 gpurun_out/upw/tests.log
timeout -k 10 120 python tools/kbench.py --ops upwarp --levels 1,2,3,4 2>/dev/null > gpurun_out/upw/kb.txt || exit 1
cat gpurun_out/upw/kb.txt
