# training-step timing of the hot path (tools/train_bench.py), then the forward bench line
set -o pipefail
mkdir -p gpurun_out/train
timeout -k 10 200 python tools/train_bench.py > gpurun_out/train/train.json 2> gpurun_out/train/train.err || { tail -20 gpurun_out/train/train.err; exit 1; }
cat gpurun_out/train/train.json
timeout -k 10 200 python bench.py --no-cpu-baseline 2>/dev/null | tail -1 > gpurun_out/train/fwd.json || exit 1
cat gpurun_out/train/fwd.json
