set -o pipefail
mkdir -p gpurun_out/g5; : > gpurun_out/g5/col.txt
timeout -k 10 60 ./tools/colbench 200 3 0 | tail -1 >> gpurun_out/g5/col.txt || exit 1
for m in 1 2 3; do
  timeout -k 10 60 ./tools/colbench_m$m 200 3 0 2>&1 | tail -1 >> gpurun_out/g5/col.txt
done
cat gpurun_out/g5/col.txt
