#!/bin/bash
# Same-box interleaved A/B of bench.py between two GEMM autotune candidate sets:
#   bash scripts/ab_tiles.sh "<DLI_GEMM_EXCLUDE of arm A>" "<DLI_GEMM_EXCLUDE of arm B>"
# e.g. "22,26" (tile 27 = the round-1 8-phase wait schedule) vs "26,27" (the default).
set -u
A=${1:-22,26}; B=${2:-26,27}
mkdir -p gpurun_out
for r in 1 2; do
  for arm in A B; do
    if [ $arm = A ]; then export DLI_GEMM_EXCLUDE="$A"; else export DLI_GEMM_EXCLUDE="$B"; fi
    timeout -k 10 300 python bench.py --steps 3 --warmup 1 > gpurun_out/abt_${arm}_$r.log 2>&1
    rc=$?; echo "rc[$arm $r exclude=$DLI_GEMM_EXCLUDE]=$rc"; grep -o '"value": [0-9.]*' gpurun_out/abt_${arm}_$r.log
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
