#!/bin/bash
# config-4 GPU tests, then the config-4 bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_config4.py > gpurun_out/t_c4.txt 2>&1 || { tail -30 gpurun_out/t_c4.txt; exit 1; }
tail -2 gpurun_out/t_c4.txt
timeout -k 10 200 python bench.py --batch 16 --height 448 --width 1024 --dtype fp16 --no-cpu-baseline --no-pmc > gpurun_out/c4b.json 2>gpurun_out/c4b.err || { tail gpurun_out/c4b.err; exit 1; }
python -c "import json; r=json.loads(open('gpurun_out/c4b.json').read().strip().splitlines()[-1]); print(r['value'], r['ms_per_step'], r['roofline']['frac'], r['checks']['replay'])"
