# corr_bwd knob A/B at l4..l2 (tools/variants.py) + census of the knob variant at l4
for l in 4 3 2; do timeout -k 10 200 python tools/variants.py --op corr_bwd --level $l --knobs "$1" || exit 1; done > gpurun_out/cbwd_ab.txt 2>&1
timeout -k 10 100 python tools/bwd_phases.py --level 4 --knobs "$1" >> gpurun_out/cbwd_ab.txt 2>&1
grep -v amdgpu.ids gpurun_out/cbwd_ab.txt | cut -c1-700
