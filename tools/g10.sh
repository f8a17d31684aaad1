set -o pipefail
mkdir -p gpurun_out/g10
for f in lds_launch_probe entry_probe launch_probe; do timeout -k 10 60 ./tools/$f > gpurun_out/g10/$f.txt 2>&1 || exit 1; done
