set -o pipefail
mkdir -p gpurun_out/g5; : > gpurun_out/g5/col.txt
for va in "0 3" "0 0"; do
  set -- $va
  timeout -k 10 60 ./tools/colbench 200 $2 $1 > gpurun_out/g5/one.txt 2>&1; rc=$?
  grep -v "^bad" gpurun_out/g5/one.txt | tail -1 >> gpurun_out/g5/col.txt
  [ $rc -eq 0 ] || exit $rc
done
