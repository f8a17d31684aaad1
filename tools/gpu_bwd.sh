# backward parity (all gradient tests) then per-level backward timings
set -o pipefail
mkdir -p gpurun_out/bwd
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests -k "backward or autograd or grad or warp" > gpurun_out/bwd/tests.log 2>&1 || { tail -40 gpurun_out/bwd/tests.log; exit 1; }
tail -3 gpurun_out/bwd/tests.log
rm -f gpurun_out/bwd/kb.txt
timeout -k 10 200 python tools/kbench.py --ops none --backward --levels 0,1,2,3,4 --tag bwd 2>/dev/null >> gpurun_out/bwd/kb.txt || exit 1
cat gpurun_out/bwd/kb.txt
