# round 4: fp32 forward warp output stores, nontemporal (tree) vs plain (build/ab_wplain): the
# warp's output is the next kernel's f2 -- bench step (dependency order) and kbench warp-then-corr
set -o pipefail
mkdir -p gpurun_out
F="--no-cpu-baseline --no-pmc --no-net-forward --no-corr4 --grouped-mode off --steps 200 --warmup 200"
for i in 1 2; do
  for v in plain tree; do
    if [ $v = plain ]; then export PWC_HOTPATH_LIB=build/ab_wplain/libpwc_hotpath.so; else unset PWC_HOTPATH_LIB; fi
    timeout -k 10 200 python bench.py $F > gpurun_out/ws_b.json 2> gpurun_out/ws_b.err || { tail gpurun_out/ws_b.err; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/ws_b.json').read().strip().splitlines()[-1]);print('$v bench', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'])"
    timeout -k 10 120 python tools/kbench.py --ops seq --levels 2,3,4 > gpurun_out/ws_k.log 2>&1 || { tail gpurun_out/ws_k.log; exit 1; }
    echo "$v seq $(grep -o '"level": [0-9].*"us": [0-9.]*' gpurun_out/ws_k.log | sed 's/"shape.*"us"/us/' | tr '\n' ' ')"
  done
done
unset PWC_HOTPATH_LIB
