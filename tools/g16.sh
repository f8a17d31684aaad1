set -o pipefail
mkdir -p gpurun_out/g16; rm -f gpurun_out/g16/var.txt
timeout -k 10 200 python tools/variants.py --op corr --level 3 --knobs "rows_r=3,rows_ts=2,rows_ck=16;rows_r=2,rows_ck=16;rows_r=3,rows_ts=3,rows_ck=32;rows_r=3,rows_ts=3,rows_ck=16;rows_r=4,rows_ts=3,rows_ck=16;rows_r=6,rows_ts=3,rows_ck=8" >> gpurun_out/g16/var.txt 2>&1 &&
timeout -k 10 200 python tools/variants.py --op corr --level 2 --knobs "rows_r=1,rows_ck=24;rows_r=1,rows_ck=96;rows_r=2,rows_ck=32;rows_r=2,rows_ts=2,rows_ck=32;rows_r=3,rows_ts=3,rows_ck=16" >> gpurun_out/g16/var.txt 2>&1
