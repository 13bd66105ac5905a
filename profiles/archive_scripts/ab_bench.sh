#!/bin/bash
# Same-box A/B of bench.py between this tree and ./ab_base (an older checkout), interleaved.
set -u
mkdir -p gpurun_out
for r in 1 2; do
  for side in base head; do
    d=.; [ $side = base ] && d=ab_base
    ( cd $d && timeout -k 10 300 python bench.py --steps 3 --warmup 1 ) > gpurun_out/ab_${side}_$r.log 2>&1
    rc=$?; echo "rc[$side $r]=$rc"; grep -o '"value": [0-9.]*' gpurun_out/ab_${side}_$r.log
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
