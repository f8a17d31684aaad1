#!/bin/bash
# GPU suite + smoke + the default bench on the current tree -> $OUT (each step under its own
# time limit; stops at the first failure)
OUT=${OUT:-gpurun_out/check}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/gputests.txt 2>&1 || { grep -E "FAIL|Error" $OUT/gputests.txt | head -20; tail -20 $OUT/gputests.txt; exit 1; }
tail -1 $OUT/gputests.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 || { tail $OUT/smoke.txt; exit 1; }
tail -1 $OUT/smoke.txt
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail $OUT/bench.err; exit 1; }
python - "$OUT/bench.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]; c = d.get("cpu_baseline", {})
print("bench", d["value"], d["ms_per_step"], "l4", r["avg_launch_us"], "frac", r["frac"], "traffic", r["traffic"],
      "cpu", c.get("value"), c.get("cores"), c.get("host_cpus"), c.get("cgroup_cpus"), c.get("lines"))
PY
