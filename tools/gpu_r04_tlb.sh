# round 4: is the strip's slowdown past ~500 MB of rotation address translation?  tools/strip_bench
# with 14 rotating sets (644 MB), the strip launch alone timed, with and without a small kernel that
# touches one dword per 64 KiB / 4 KiB of that launch's buffers first (STRIP_WARM)
set -o pipefail
for i in 1 2; do
  for w in 0 65536 4096; do
    echo "sets=14 warm=$w $(STRIP_SETS=14 STRIP_WARM=$w timeout -k 10 60 tools/strip_bench 300 | tail -1)"
  done
  echo "sets=2 warm=0 $(STRIP_SETS=2 timeout -k 10 60 tools/strip_bench 300 | tail -1)"
done
