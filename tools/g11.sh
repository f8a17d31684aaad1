set -o pipefail
mkdir -p gpurun_out/g11; : > gpurun_out/g11/var.txt
for lv in 2 3 4; do
timeout -k 10 120 python tools/variants.py --op warp_bwd --level $lv >> gpurun_out/g11/var.txt 2>&1 || exit 1
timeout -k 10 120 python tools/variants.py --op corr_bwd --level $lv >> gpurun_out/g11/var.txt 2>&1 || exit 1
done
