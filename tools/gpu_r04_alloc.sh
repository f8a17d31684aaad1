# round 4: does the allocator's segment mapping change the bench step (l4 in-step time)?
# default caching allocator vs expandable segments (hipMemCreate/hipMemMap), alternating.
set -o pipefail
F="--no-cpu-baseline --no-pmc --no-net-forward --no-corr4 --grouped-mode off --steps 200 --warmup 200"
for run in 1 2; do
  for conf in default expandable_segments:True; do
    if [ $conf = default ]; then unset PYTORCH_HIP_ALLOC_CONF; else export PYTORCH_HIP_ALLOC_CONF=$conf; fi
    timeout -k 10 200 python bench.py $F > gpurun_out/alloc_b.json 2> gpurun_out/alloc_b.err || { tail gpurun_out/alloc_b.err; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/alloc_b.json').read().strip().splitlines()[-1]);print('$conf', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'])"
  done
done
