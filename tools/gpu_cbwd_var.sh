# correlation backward variants: band height / channels per item (PWC_BWD_CFG), slices
set -o pipefail
mkdir -p gpurun_out/cbv; rm -f gpurun_out/cbv/kb.txt
timeout -k 10 100 python tools/kbench.py --ops none --backward --levels 0,1,2,3,4 --tag "auto" 2>/dev/null | grep corr_bwd >> gpurun_out/cbv/kb.txt || exit 1
for v in "3,4" "2,4" "1,4" "3,2" "3,8"; do
  PWC_BWD_CFG=$v timeout -k 10 100 python tools/kbench.py --ops none --backward --levels 2,3,4 --tag "cfg$v" 2>/dev/null | grep corr_bwd >> gpurun_out/cbv/kb.txt || exit 1
done
for v in 1 2 4; do
  PWC_BWD_SLICES=$v timeout -k 10 100 python tools/kbench.py --ops none --backward --levels 3,4 --tag "sl$v" 2>/dev/null | grep corr_bwd >> gpurun_out/cbv/kb.txt || exit 1
done
python3 -c "
import json
for l in open('gpurun_out/cbv/kb.txt'):
    d=json.loads(l); print(d['level'], d['op'], d.get('tag',''), d['us'])"
