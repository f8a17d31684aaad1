# round 4: ablations of the fp16 strip kernel (census build, knob s16_abl: 1 no reads/dots,
# 2 no stores, 4 no loader staging after the first barrier), config-4 l4
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 60 python tools/kbench.py --batch 16 --height 448 --width 1024 --dtype fp16 --levels 4 --ops corr > gpurun_out/s16prod.log 2>&1 || exit 1; echo "prod $(tail -1 gpurun_out/s16prod.log)"
for a in 0 1 2 4 3 5 6 7 0; do
  PWC_HOTPATH_LIB=build/census/libpwc_hotpath.so PWC_DEBUG=s16_abl=$a timeout -k 10 60 python tools/kbench.py --batch 16 --height 448 --width 1024 --dtype fp16 --levels 4 --ops corr > gpurun_out/s16abl_$a.log 2>&1 || exit 1
  echo "abl=$a $(tail -1 gpurun_out/s16abl_$a.log)"
done
