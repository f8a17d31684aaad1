#!/bin/bash
# grouped l0 + l1 launch: parity tests, bench A/B (group on / off, alternating), kernel trace
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/grp
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/grp/pytest.txt 2>&1; rc=$?; tail -3 gpurun_out/grp/pytest.txt; [ $rc -eq 0 ] || exit 1
for i in 1 2 3; do
  for g in on off; do
    timeout -k 10 120 python bench.py --group $g --no-cpu-baseline --no-pmc > gpurun_out/grp/b_$g$i.json 2> gpurun_out/grp/b_$g$i.err || { tail gpurun_out/grp/b_$g$i.err; exit 1; }
    python -c "import json,sys; d=json.load(open('gpurun_out/grp/b_$g$i.json')); print('$g', d['value'], d['ms_per_step'], d['roofline']['frac'], d['checks']['replay'])"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/grp/prof -o run --output-format csv -- python bench.py --no-cpu-baseline --no-pmc --steps 200 > gpurun_out/grp/prof.log 2>&1 || { tail gpurun_out/grp/prof.log; exit 1; }
python - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/grp/prof/**/run_kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:9]:
    print(r["Calls"], round(float(r["AverageNs"])/1000, 2), r["Name"][:90])
PY
