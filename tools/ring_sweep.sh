#!/bin/bash
# Times the correlation forward per pyramid level for ring configurations (PWC_RING_CFG).
set -o pipefail
CFGS=${CFGS:-"A B C D E F G H I"}
for cfg in $CFGS; do
  PWC_RING_CFG=$cfg timeout -k 10 120 python tools/kbench.py --levels ${LEVELS:-2,3,4} --iters 40 2>/dev/null | grep corr_fwd | sed "s/^/$cfg /" || exit 1
done
