set -o pipefail
mkdir -p gpurun_out/g22; rm -f gpurun_out/g22/var.txt
for lv in 2 3; do timeout -k 10 200 python tools/variants.py --op corr --level $lv --knobs "corr_band=2;corr_band=2,band_r=2,band_t=3;corr_band=2,band_r=1,band_t=3;corr_band=2,band_r=3,band_t=1" >> gpurun_out/g22/var.txt 2>&1 || exit 1; done
for lv in 2 3 4; do timeout -k 10 200 python tools/variants.py --op corr_bwd --level $lv --knobs "bwd_ct=4;bwd_r=2;bwd_r=2,bwd_ct=4;bwd_slices=2" >> gpurun_out/g22/var.txt 2>&1 || exit 1; done
