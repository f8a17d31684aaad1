#!/bin/bash
# correlation-backward phase census (library built with `make CENSUS=1`) at l4 and l3
# (one configuration: the three-tj variant the old A/B compared against was removed in round 3)
set -o pipefail
for l in 4 3; do timeout -k 10 100 python tools/bwd_phases.py --level $l || exit 1; done 2>&1 | grep -v amdgpu.ids
