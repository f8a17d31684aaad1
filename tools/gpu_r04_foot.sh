# round 4: l4 strip vs stream kernel time against the rotating footprint (tools/strip_bench, sets
# of 46 MB each) and the bench with 3 / 4 sets
set -o pipefail
for n in 1 2 7 14 24; do echo "sets=$n $(STRIP_SETS=$n timeout -k 10 60 tools/strip_bench 300 | tail -1)"; done
F="--no-cpu-baseline --no-pmc --no-net-forward --no-corr4 --grouped-mode off --steps 100 --warmup 100"
for s in 3 4 12; do
  timeout -k 10 200 python bench.py $F --sets $s > gpurun_out/sets_b.json 2> gpurun_out/sets_b.err || { tail gpurun_out/sets_b.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/sets_b.json').read().strip().splitlines()[-1]);print('bench sets=$s', d['ms_per_step'], d['roofline']['avg_launch_us'])"
done
