# round 4: does the l4 strip correlation's in-step time depend on the bench's buffer-set rotation?
set -o pipefail
mkdir -p gpurun_out/sets
F="--no-cpu-baseline --no-pmc --no-net-forward --no-corr4 --grouped-mode off --steps 100 --warmup 100"
for s in 1 2 0; do
  timeout -k 10 200 python bench.py $F --sets $s > gpurun_out/sets/b$s.json 2> gpurun_out/sets/b$s.err || { tail gpurun_out/sets/b$s.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/sets/b$s.json').read().strip().splitlines()[-1]);print('sets=$s', d['config']['buffer_sets'], d['ms_per_step'], d['roofline']['avg_launch_us'])"
done
PWC_DEBUG=strip=0 timeout -k 10 200 python bench.py $F > gpurun_out/sets/bs.json 2> gpurun_out/sets/bs.err || exit 1
python -c "import json;d=json.loads(open('gpurun_out/sets/bs.json').read().strip().splitlines()[-1]);print('strip=0', d['config']['buffer_sets'], d['ms_per_step'], d['roofline']['avg_launch_us'])"
timeout -k 10 100 python tools/kbench.py --levels 4 --ops corr --sets 1 | grep level
timeout -k 10 100 python tools/kbench.py --levels 4 --ops corr | grep level
