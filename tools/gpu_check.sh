#!/bin/bash
# full GPU tests + smoke, then the default bench, the graph-all comparison and the train step
set -o pipefail
bash tools/gpu_tests.sh || exit 1
mkdir -p gpurun_out/b
timeout -k 10 400 python bench.py --steps 200 --warmup 20 --cpu-seconds 5 > gpurun_out/b/bench.json 2> gpurun_out/b/bench.err || { tail -5 gpurun_out/b/bench.err; exit 1; }
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-pmc --timing graph-all > gpurun_out/b/bench_all.json 2> gpurun_out/b/bench_all.err || exit 1
timeout -k 10 300 python bench.py --dtype fp16 --batch 16 --height 448 --width 1024 --steps 100 --warmup 10 --no-cpu-baseline --no-pmc > gpurun_out/b/cfg4.json 2> gpurun_out/b/cfg4.err || exit 1
timeout -k 10 200 python tools/train_bench.py > gpurun_out/b/train.json 2> gpurun_out/b/train.err || exit 1
python - <<'PY'
import json
for f in ["bench", "bench_all", "cfg4", "train"]:
    d = json.loads(open(f"gpurun_out/b/{f}.json").read().strip().splitlines()[-1])
    print(f, d["value"], d["ms_per_step"], d.get("roofline", {}).get("avg_launch_us"), d.get("roofline", {}).get("frac"), d.get("checks", {}).get("replay"))
PY
