# training step (JSON) -> gpurun_out/train_q.json, summary line
set -o pipefail
timeout -k 10 300 python tools/train_bench.py > gpurun_out/train_q.json 2> gpurun_out/train_q.err || { tail gpurun_out/train_q.err; exit 1; }
python - <<'PY'
import json
t = json.load(open("gpurun_out/train_q.json"))
print(t["ms_per_step"], t["checks"]["self_check"]["ok"], t["grouped"]["ms_per_step"])
for r in t["kernels"]:
    print(r["level"], r["op"], r["us"], r["frac_8TBs"])
PY
