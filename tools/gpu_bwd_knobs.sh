#!/bin/bash
set -o pipefail
for l in 4 3 2; do
timeout -k 10 200 python tools/variants.py --op warp_bwd --level $l --knobs "warp_tiles=2;warp_tiles=2,warp_bwd_ng=2;warp_tiles=2,warp_bwd_ng=4;warp_bwd_ng=2;warp_tiles=3" 2>&1 | grep us
timeout -k 10 200 python tools/variants.py --op corr_bwd --level $l --knobs "bwd_slices=2;bwd_slices=3;bwd_r=2;bwd_r=1" 2>&1 | grep us
done
