set -o pipefail
mkdir -p gpurun_out/g6; : > gpurun_out/g6/s.txt
for v in 0 64 0 64; do
  echo -n "stream_abl=$v " >> gpurun_out/g6/s.txt
  PWC_DEBUG=stream_abl=$v timeout -k 10 60 ./tools/sbench 200 >> gpurun_out/g6/s.txt 2>&1 || exit 1
done
cat gpurun_out/g6/s.txt
