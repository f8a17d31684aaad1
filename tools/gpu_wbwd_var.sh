# warp backward tile-shape variants (PWC_WARP_TILES) and flow magnitudes, l2/l4
set -o pipefail
mkdir -p gpurun_out/wbv; rm -f gpurun_out/wbv/kb.txt
for v in 0 1 2 3 4; do
  PWC_WARP_TILES=$v timeout -k 10 100 python tools/kbench.py --ops none --backward --levels 2,4 --tag "t$v" 2>/dev/null | grep warp_bwd >> gpurun_out/wbv/kb.txt || exit 1
done
PWC_WARP_TILES=0 timeout -k 10 100 python tools/kbench.py --ops none --backward --levels 2,4 --flow-scale 0 --tag "t1fs0" 2>/dev/null | grep warp_bwd >> gpurun_out/wbv/kb.txt || exit 1
PWC_WARP_TILES=0 PWC_WARP_BWD_NG=16 timeout -k 10 100 python tools/kbench.py --ops none --backward --levels 2,4 --tag "t1ng16" 2>/dev/null | grep warp_bwd >> gpurun_out/wbv/kb.txt || exit 1
cat gpurun_out/wbv/kb.txt
