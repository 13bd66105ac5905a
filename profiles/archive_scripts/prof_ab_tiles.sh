#!/bin/bash
# rocprofv3 kernel summaries of one bench wave with tile 26 excluded / allowed (A/B of a tile
# in situ: the per-kernel times of the same decode GEMMs under both plans).
set -u
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for side in no26 with26; do
  if [ $side = no26 ]; then export DLI_GEMM_EXCLUDE=26; else export DLI_GEMM_EXCLUDE=" "; fi
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$side -o bench -- python bench.py --steps 1 --warmup 1 > gpurun_out/prof_$side.log 2>&1 || exit $?
  python scripts/prof_summary.py gpurun_out/prof_$side 14 --tail-ms 900 > gpurun_out/prof_${side}_summary.txt
  rm -f gpurun_out/prof_$side/*trace.csv
  head -12 gpurun_out/prof_${side}_summary.txt | cut -c1-110
done
