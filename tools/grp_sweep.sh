#!/bin/bash
# Times the correlation forward at the coarse levels per coarse-kernel configuration
# (PWC_GRP_CFG) and with the coarse kernel disabled (split path).
set -o pipefail
for cfg in ${CFGS:-A B C D E}; do
  PWC_GRP_CFG=$cfg timeout -k 10 120 python tools/kbench.py --levels ${LEVELS:-0,1,2,3} --iters 40 2>/dev/null | grep corr_fwd | sed "s/^/$cfg /" || exit 1
done
PWC_CORR_GRP=0 timeout -k 10 120 python tools/kbench.py --levels ${LEVELS:-0,1,2,3} --iters 40 2>/dev/null | grep corr_fwd | sed "s/^/split /" || exit 1
