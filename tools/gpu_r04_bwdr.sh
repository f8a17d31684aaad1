# round 4: correlation backward band height (knob bwd_r) at l2..l4, config 5 shapes
set -o pipefail
for k in default bwd_r=4 bwd_r=5 bwd_r=6 default; do
  PWC_DEBUG=$([ $k = default ] || echo $k) timeout -k 10 120 python tools/kbench.py --levels 2,3,4 --ops none --backward > gpurun_out/bwdr.log 2>&1 || exit 1
  echo "$k $(grep corr_bwd gpurun_out/bwdr.log | python -c 'import sys,json;print([(json.loads(l)["level"], json.loads(l)["us"]) for l in sys.stdin])')"
done
