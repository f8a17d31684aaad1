#!/bin/bash
# full GPU tests + smoke, then the default bench (graph-eager) and the graph-all comparison
set -o pipefail
bash tools/gpu_tests.sh || exit 1
mkdir -p gpurun_out/b
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --cpu-seconds 5 > gpurun_out/b/bench.json 2> gpurun_out/b/bench.err || { tail -5 gpurun_out/b/bench.err; exit 1; }
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --timing graph-all > gpurun_out/b/bench_all.json 2> gpurun_out/b/bench_all.err || exit 1
python - <<'PY'
import json
for f in ["bench", "bench_all"]:
    d = json.loads(open(f"gpurun_out/b/{f}.json").read().strip().splitlines()[-1])
    print(f, d["value"], d["ms_per_step"], d.get("roofline", {}).get("avg_launch_us"), d["checks"]["replay"])
PY
