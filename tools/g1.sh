set -o pipefail
mkdir -p gpurun_out/g1
timeout -k 10 60 ./tools/issue_probe > gpurun_out/g1/issue.txt 2>&1 && \
timeout -k 10 60 ./tools/sbench 100 > gpurun_out/g1/sbench.txt 2>&1 && \
timeout -k 10 300 python bench.py --no-pmc --no-cpu-baseline > gpurun_out/g1/bench.json 2> gpurun_out/g1/bench.err && \
timeout -k 10 300 python bench.py --no-pmc --no-cpu-baseline --group off --corr-group off --warp-group off > gpurun_out/g1/bench_nogroup.json 2> gpurun_out/g1/bench_nogroup.err
echo rc=$?
cat gpurun_out/g1/issue.txt gpurun_out/g1/sbench.txt
