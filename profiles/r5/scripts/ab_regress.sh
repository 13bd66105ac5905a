#!/bin/bash
# Same-box A/B of the driver's exact bench command: round-3 HEAD (./ab_base, e66238d) vs this
# tree, alternated 3x. One JSON line per run into gpurun_out/ab_regress.jsonl.
set -u
mkdir -p gpurun_out
out=gpurun_out/ab_regress.jsonl
: > $out
for r in 1 2 3; do
  for side in r3 head; do
    d=.; [ $side = r3 ] && d=ab_base
    log=gpurun_out/ab_${side}_$r.log
    ( cd $d && timeout -k 10 240 python3 bench.py --gpus 1 --steps 20 --warmup 5 ) > $log 2>&1
    rc=$?
    echo "rc[$side $r]=$rc"
    [ $rc -ne 0 ] && { tail -20 $log; exit $rc; }
    line=$(grep '^{"metric"' $log)
    echo "{\"side\": \"$side\", \"run\": $r, \"bench\": $line}" >> $out
    echo "$side $r $(echo "$line" | grep -o '"value": [0-9.]*')"
  done
done
exit 0
