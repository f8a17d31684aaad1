set -o pipefail
mkdir -p gpurun_out/g9; : > gpurun_out/g9/var.txt
for lv in 2 4; do
  timeout -k 10 120 python tools/variants.py --op warp --level $lv --knobs "warp_rows=0;warp_rows_abl=1;warp_rows_abl=2;warp_rows_abl=4;warp_rows_abl=6;warp_rows_abl=7" >> gpurun_out/g9/var.txt 2>&1 || exit 1
done
