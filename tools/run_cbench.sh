#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/cb2
timeout -k 10 120 ./tools/cbench 8 32 96 112 200 > gpurun_out/cb2/l4.txt 2>&1 || exit 1
NSETS=1 timeout -k 10 120 ./tools/cbench 8 32 96 112 200 > gpurun_out/cb2/l4_ns1.txt 2>&1 || exit 1
PWC_PAR_CFG=B ONLY=par timeout -k 10 120 ./tools/cbench 8 32 96 112 200 > gpurun_out/cb2/l4_B.txt 2>&1 || exit 1
echo ok
