#!/bin/bash
# bench in both timing modes (graph = whole step in per-step graphs with event nodes;
# graph-eager = round-2 measurement) -> gpurun_out/modes
set -o pipefail
OUT=gpurun_out/modes; mkdir -p $OUT
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --timing graph-all > $OUT/graph.json 2> $OUT/graph.err || { tail -20 $OUT/graph.err; exit 1; }
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --timing graph-eager > $OUT/ge.json 2> $OUT/ge.err || { tail -20 $OUT/ge.err; exit 1; }
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python bench.py --steps 200 --warmup 20 --no-cpu-baseline > $OUT/traced.json 2> $OUT/trace.err || exit 1
python - <<'PY'
import json
for f in ["graph","ge","traced"]:
    d=json.loads(open(f"gpurun_out/modes/{f}.json").read().strip().splitlines()[-1])
    print(f, d["value"], d["ms_per_step"], d.get("roofline",{}).get("avg_launch_us"), d["checks"]["replay"])
PY
