set -o pipefail
mkdir -p gpurun_out/g7
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_train_step.py tests/test_pred.py > gpurun_out/g7/tests.txt 2>&1 &&
timeout -k 10 300 python bench.py --no-cpu-baseline --no-pmc > gpurun_out/g7/bench.json 2> gpurun_out/g7/bench.err &&
timeout -k 10 300 python tools/train_bench.py > gpurun_out/g7/train.json 2> gpurun_out/g7/train.err
rc=$?
tail -3 gpurun_out/g7/tests.txt; exit $rc
