#!/bin/bash
# config 4 (fp16 448x1024, B=16): fp16 parity tests, l4/l3 correlation times, the config-4 bench
set -o pipefail
mkdir -p gpurun_out
PWC_DEBUG=stream_abl=64 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_config4.py tests/test_gpu_parity.py -k "fp16 or half or config4 or sintel or stress or Sintel" > gpurun_out/cfg4_tests.txt 2>&1 || { tail -30 gpurun_out/cfg4_tests.txt; exit 1; }
tail -1 gpurun_out/cfg4_tests.txt
for l in 4 3; do timeout -k 10 200 python tools/variants.py --op corr --level $l --dtype fp16 --batch 16 --height 448 --width 1024 --knobs "stream_abl=64;stream_abl=65;stream_abl=66" 2>&1 | grep us | cut -c1-120 || exit 1; done
PWC_DEBUG=stream_abl=64 timeout -k 10 300 python bench.py --dtype fp16 --batch 16 --height 448 --width 1024 --no-cpu-baseline > gpurun_out/cfg4_ab.json 2> gpurun_out/cfg4_ab.err || { tail gpurun_out/cfg4_ab.err; exit 1; }
python -c "import json; c=json.load(open('gpurun_out/cfg4_ab.json')); print('cfg4', c['value'], c['ms_per_step'], c['roofline']['frac'], c['roofline']['avg_launch_us'])"
