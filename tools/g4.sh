set -o pipefail
mkdir -p gpurun_out/g4
timeout -k 10 60 ./tools/colbench 200 > gpurun_out/g4/col.txt 2>&1; rc=$?
cat gpurun_out/g4/col.txt
exit $rc
