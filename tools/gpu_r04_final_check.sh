# round 4 close: the GPU suite, smoke and the default bench on the final tree (no profiler)
set -o pipefail
mkdir -p gpurun_out/final
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/ > gpurun_out/final/gputests.txt 2>&1 || { tail -30 gpurun_out/final/gputests.txt; exit 1; }
tail -1 gpurun_out/final/gputests.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final/smoke.txt 2>&1 || { tail gpurun_out/final/smoke.txt; exit 1; }
tail -1 gpurun_out/final/smoke.txt
timeout -k 10 600 python bench.py > gpurun_out/final/bench.json 2> gpurun_out/final/bench.err || { tail gpurun_out/final/bench.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/final/bench.json').read().strip().splitlines()[-1]);print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['avg_launch_us'])"
