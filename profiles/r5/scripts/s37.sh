#!/bin/bash
# Session 37: batch-1 sampler chunk count (DLI_SAMPLE_PMAX 32 vs the default 64), alternated.
set -u
O=gpurun_out/s37
mkdir -p $O
: > $O/ab.jsonl
run() { local name=$1; shift; echo "== $name"; timeout -k 10 240 "$@" > $O/$name.log 2>&1; local rc=$?;
        echo "rc[$name]=$rc"; [ $rc -eq 0 ] || exit $rc;
        echo "{\"arm\": \"$name\", \"bench\": $(grep -h '^{"metric"' $O/$name.log)}" >> $O/ab.jsonl; }
for i in 1 2; do
  run p64_$i python3 bench.py --batch 1 --steps 8 --warmup 2
  run p32_$i env DLI_SAMPLE_PMAX=32 python3 bench.py --batch 1 --steps 8 --warmup 2
done
exit 0
