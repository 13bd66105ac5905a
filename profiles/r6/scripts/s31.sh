#!/bin/bash
# Session 31 (round 6): hardware counters of the headline wave on the final HEAD —
# scripts/pmc.sh over `bench.py --steps 1 --warmup 1` (five --pmc passes, each alone, each
# under its own SIGKILL timeout), the per-kernel report over the last wave's dispatches
# (PMC_TAIL = one wave of the Llama-3-8B b512 bench: 16,471 dispatches, s30).
set -u
O=gpurun_out/r6s31
mkdir -p $O
PMC_TAIL=16471 bash scripts/pmc.sh $O/pmc
rc=$?; echo "rc[pmc]=$rc"
for d in $O/pmc/pass*; do [ -d "$d" ] && rm -rf "$d"; done
exit $rc
