set -o pipefail
mkdir -p gpurun_out/g21; rm -f gpurun_out/g21/var.txt
timeout -k 10 300 python tools/variants.py --op corr --level 4 --dtype fp16 --batch 16 --height 448 --width 1024 --knobs "stream_abl=1;stream_abl=4;stream_abl=5;stream_abl=2;stream_abl=3;stream_abl=7" >> gpurun_out/g21/var.txt 2>&1
