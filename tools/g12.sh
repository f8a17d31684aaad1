set -o pipefail
mkdir -p gpurun_out/g12; : > gpurun_out/g12/var.txt
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "warp_backward" > gpurun_out/g12/tests.txt 2>&1; rc=$?
tail -30 gpurun_out/g12/tests.txt
[ $rc -eq 0 ] || exit $rc
for lv in 0 1 2 3 4; do
timeout -k 10 120 python tools/variants.py --op warp_bwd --level $lv --knobs "warp_bwd_tiles=0" >> gpurun_out/g12/var.txt 2>&1 || exit 1
done
