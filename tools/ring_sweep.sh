#!/bin/bash
# Times the correlation forward per pyramid level for every ring configuration (PWC_RING_CFG).
set -o pipefail
for cfg in A B C D E; do
  PWC_RING_CFG=$cfg timeout -k 10 120 python tools/kbench.py --levels 2,3,4 --iters 40 2>/dev/null | grep corr_fwd | sed "s/^/$cfg /" || exit 1
done
