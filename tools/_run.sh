set -o pipefail
mkdir -p gpurun_out/cb9
ONLY=pt timeout -k 10 120 ./tools/cbench 8 32 96 112 200 > gpurun_out/cb9/l4.txt 2>&1 || exit 1
ONLY=grp timeout -k 10 120 ./tools/cbench 8 64 48 56 200 > gpurun_out/cb9/l3_grp.txt 2>&1 || exit 1
for k in 2 4 8; do PWC_PT_K=$k ONLY=pt timeout -k 10 120 ./tools/cbench 8 64 48 56 200 > gpurun_out/cb9/l3_$k.txt 2>&1 || exit 1; done
ONLY=grp timeout -k 10 120 ./tools/cbench 8 96 24 28 200 > gpurun_out/cb9/l2_grp.txt 2>&1 || exit 1
for k in 4 8; do PWC_PT_K=$k ONLY=pt timeout -k 10 120 ./tools/cbench 8 96 24 28 200 > gpurun_out/cb9/l2_$k.txt 2>&1 || exit 1; done
