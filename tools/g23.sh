set -o pipefail
mkdir -p gpurun_out/g23
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "warp" > gpurun_out/g23/tests.txt 2>&1 || { tail -30 gpurun_out/g23/tests.txt; exit 1; }
tail -1 gpurun_out/g23/tests.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/g23/tt -o run --output-format csv -- python tools/train_bench.py --grouped-mode off --no-kernels > gpurun_out/g23/train.json 2> gpurun_out/g23/train.err
