#!/bin/bash
# round 4, session 29: PMC counter passes over one decode layer's kernels at batch 512
# (scripts/pmc.sh -> pmc_decode_ops.py) with the round-4 plans
set -o pipefail
bash scripts/pmc.sh && mkdir -p gpurun_out/r4s29 && cp -r gpurun_out/pmc/*.txt gpurun_out/pmc/*.log gpurun_out/pmc/*.json gpurun_out/r4s29/ 2>/dev/null
rm -rf gpurun_out/pmc/pass*
