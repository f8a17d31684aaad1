#!/bin/bash
# correlation-backward phase census (library built with `make CENSUS=1`): TG = 3 vs TG = 1
set -o pipefail
for k in "" "bwd_tg=1"; do
for l in 4 3; do timeout -k 10 100 python tools/bwd_phases.py --level $l --knobs "$k" || exit 1; done 2>&1 | grep -v amdgpu.ids
done
