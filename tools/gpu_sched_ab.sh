#!/bin/bash
# A/B of two builds of the standalone l4 stream-correlation bench (tools/sbench.hip)
set -o pipefail
for i in 1 2 3; do for b in base sched; do
  echo -n "$b "; timeout -k 10 60 ./tools/sbench_$b 200 || exit 1
done; done
