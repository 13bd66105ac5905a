#!/bin/bash
# Same-box interleaved A/B of bench.py with tile 26 kept out of / allowed in the GEMM autotune.
set -u
for r in 1 2; do
  for side in no26 with26; do
    if [ $side = no26 ]; then export DLI_GEMM_EXCLUDE=26; else export DLI_GEMM_EXCLUDE=" "; fi
    timeout -k 10 300 python bench.py --steps 3 --warmup 1 > gpurun_out/ab26_${side}_$r.log 2>&1
    rc=$?; echo "rc[$side $r]=$rc"; grep -o '"value": [0-9.]*' gpurun_out/ab26_${side}_$r.log
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
