set -o pipefail
mkdir -p gpurun_out/g20; rm -f gpurun_out/g20/var2.txt
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_config4.py tests/test_gpu_fused.py > gpurun_out/g20/tests.txt 2>&1 || { tail -40 gpurun_out/g20/tests.txt; exit 1; }
tail -1 gpurun_out/g20/tests.txt
for lv in 0 1; do timeout -k 10 200 python tools/variants.py --op warp_corr --level $lv --dtype fp16 --batch 16 --height 448 --width 1024 --knobs "fused=0" >> gpurun_out/g20/var2.txt 2>&1 || exit 1; done
timeout -k 10 300 python bench.py --no-cpu-baseline --no-pmc --dtype fp16 --batch 16 --height 448 --width 1024 --steps 100 > gpurun_out/g20/cfg4.json 2> gpurun_out/g20/cfg4.err
timeout -k 10 300 python bench.py --no-cpu-baseline --no-pmc --dtype fp16 --batch 16 --height 448 --width 1024 --steps 100 --fused-levels 1 > gpurun_out/g20/cfg4_nofuse.json 2> gpurun_out/g20/cfg4.err
