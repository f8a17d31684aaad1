set -o pipefail
mkdir -p gpurun_out/s11
for sp in 4 8 16; do PWC_SMALL_SPLITS=$sp timeout -k 10 120 python tools/kbench.py --levels 0,1 --iters 60 2>/dev/null | grep corr_fwd | sed "s/^/$sp /" >> gpurun_out/s11/sweep.txt || exit 1; done
