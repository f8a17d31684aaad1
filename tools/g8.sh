set -o pipefail
mkdir -p gpurun_out/g8
export TMPDIR=/tmp
timeout -k 10 300 python tools/train_bench.py --grouped-mode off > gpurun_out/g8/train.json 2> gpurun_out/g8/train.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/g8/pb -o run --output-format csv -- python bench.py --no-cpu-baseline --no-pmc --grouped-mode off --steps 200 > gpurun_out/g8/bench.json 2> gpurun_out/g8/bench.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/g8/pt -o run --output-format csv -- python tools/train_bench.py --grouped-mode off --no-kernels > gpurun_out/g8/train2.json 2> gpurun_out/g8/train2.err
