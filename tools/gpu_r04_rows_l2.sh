# round 4: l2 row-band correlation with 1-row bands split by displacement rows (384 / 576
# workgroups instead of 192) -- tools/variants.py, event time per op and max diff to default
set -o pipefail
timeout -k 10 200 python tools/variants.py --op corr --level 2 --knobs "rows_r=1,rows_ts=2,rows_ck=48;rows_r=1,rows_ts=3,rows_ck=48;rows_r=1,rows_ts=2,rows_ck=96;rows_r=1,rows_ts=3,rows_ck=96;rows_r=1,rows_ts=9,rows_ck=96" > gpurun_out/rows_l2.txt 2>&1 || { tail gpurun_out/rows_l2.txt; exit 1; }
cat gpurun_out/rows_l2.txt
