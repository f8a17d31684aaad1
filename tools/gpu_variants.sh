# kernel-variant sweep: warp configurations (PWC_WARP_CFG) and the band kernel as plain
# correlation (PWC_CORR_BAND=1, PWC_BAND_CFG) per level, graph-timed (tools/kbench.py)
set -o pipefail
mkdir -p gpurun_out/var
for w in 0 1 2 4 5 6 7 9; do
  PWC_WARP_CFG=$w timeout -k 10 120 python tools/kbench.py --ops warp --levels 2,3,4 --tag "warp$w" 2>/dev/null >> gpurun_out/var/kb.txt || exit 1
done
timeout -k 10 120 python tools/kbench.py --ops corr --levels 0,1,2,3 --tag "corr-default" 2>/dev/null >> gpurun_out/var/kb.txt || exit 1
for c in "3,1" "2,3" "3,3" "4,3" "2,1" "4,1"; do
  PWC_CORR_BAND=1 PWC_BAND_CFG=$c timeout -k 10 120 python tools/kbench.py --ops corr --levels 0,1,2,3 --tag "band$c" 2>/dev/null >> gpurun_out/var/kb.txt || exit 1
done
cat gpurun_out/var/kb.txt | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['level'], d['op'], d['tag'], d['us'])"
