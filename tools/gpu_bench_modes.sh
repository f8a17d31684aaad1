#!/bin/bash
# bench.py timing modes side by side (value, ms/step, host issue ms/step, l4 event us, replay)
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/modes
for mode in eager graph-eager graph-all eager; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-pmc --timing $mode $EXTRA > gpurun_out/modes/$mode.json 2> gpurun_out/modes/$mode.err || { tail gpurun_out/modes/$mode.err; exit 1; }
  python -c "import json,sys; r=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], r['value'], r['ms_per_step'], r['host_issue_ms_per_step'], r.get('roofline',{}).get('avg_launch_us'), r['checks']['replay'])" gpurun_out/modes/$mode.json $mode
done
