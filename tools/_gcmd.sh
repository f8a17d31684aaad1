set -o pipefail
for a in 0 1 2; do timeout -k 10 60 ./tools/occ_m0 8 $a 32 96 112 1 | grep -v Ring || exit 1; done
