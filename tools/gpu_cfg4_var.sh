set -o pipefail
mkdir -p gpurun_out/var
for lv in 4 3; do
timeout -k 10 200 python tools/variants.py --op corr --level $lv --batch 16 --height 448 --width 1024 --dtype fp16 --knobs "stream_r=2;stream_r=4;stream_r=5" > gpurun_out/var/cfg4_l$lv.txt 2>&1 || { tail -5 gpurun_out/var/cfg4_l$lv.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/var/cfg4_l$lv.txt | cut -c1-200
done
