# round 4: strip kernel with two loader waves (whole window in flight): parity tests, standalone
# timing, then the bench step A/B against the one-loader build (build/ab_old) on the same box
set -o pipefail
mkdir -p gpurun_out/s2
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_coverage.py tests/test_gpu_parity.py > gpurun_out/s2/t.log 2>&1; rc=$?; tail -3 gpurun_out/s2/t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 60 tools/strip_bench 300 | tail -2
F="--no-cpu-baseline --no-pmc --no-net-forward --no-corr4 --grouped-mode off --steps 200 --warmup 200"
for i in 1 2; do
  timeout -k 10 200 python bench.py $F > gpurun_out/s2/new.json 2> gpurun_out/s2/new.err || { tail gpurun_out/s2/new.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/s2/new.json').read().strip().splitlines()[-1]);print('two loaders', d['ms_per_step'], d['roofline']['avg_launch_us'])"
  PWC_HOTPATH_LIB=build/ab_old/libpwc_hotpath.so timeout -k 10 200 python bench.py $F > gpurun_out/s2/old.json 2> gpurun_out/s2/old.err || { tail gpurun_out/s2/old.err; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/s2/old.json').read().strip().splitlines()[-1]);print('one loader ', d['ms_per_step'], d['roofline']['avg_launch_us'])"
done
# ablations of the matrix-core strip kernel (census build, knob ms_abl: 1 no reads/MFMA/diagonals,
# 2 no stores, 4 no loader staging after step 0), config-4 l4 and l3
for a in 0 1 2 4 3 6 5 7; do
  PWC_HOTPATH_LIB=build/census/libpwc_hotpath.so PWC_DEBUG=ms_abl=$a timeout -k 10 60 python tools/kbench.py --batch 16 --height 448 --width 1024 --dtype fp16 --levels 3,4 --ops corr > gpurun_out/s2/abl_$a.log 2>&1 || exit 1
  echo "ms_abl=$a $(grep corr_fwd gpurun_out/s2/abl_$a.log | python -c 'import sys,json;print([(json.loads(l)["level"], json.loads(l)["us"]) for l in sys.stdin])')"
done
