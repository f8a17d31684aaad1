set -o pipefail
mkdir -p gpurun_out/g13; rm -f gpurun_out/g13/ph.txt gpurun_out/g13/var.txt
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "warp_backward" > gpurun_out/g13/tests.txt 2>&1 || { tail -30 gpurun_out/g13/tests.txt; exit 1; }
tail -2 gpurun_out/g13/tests.txt
for l in 0 2 3 4; do timeout -k 10 100 python tools/wbwd_phases.py --level $l >> gpurun_out/g13/ph.txt 2>&1 || exit 1; done
for lv in 0 1 2 3 4; do
timeout -k 10 120 python tools/variants.py --op warp_bwd --level $lv --knobs "warp_bwd_tiles=0" >> gpurun_out/g13/var.txt 2>&1 || exit 1
done
