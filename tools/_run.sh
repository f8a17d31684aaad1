set -o pipefail
mkdir -p gpurun_out/cb7
for c in A B C; do PWC_PT_CFG=$c ONLY=pt timeout -k 10 120 ./tools/cbench 8 32 96 112 200 > gpurun_out/cb7/l4_$c.txt 2>&1 || exit 1; done
