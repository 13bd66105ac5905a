#!/bin/bash
# Session 21: decode attention forms at batch 512, same box, alternated: the default fused
# one-wave-per-item kernel vs a workgroup per item (DLI_DECODE_WPI=4) vs the pipelined
# (unfused) kernel (DLI_DECODE_PIPE=1). 10 timed steps each.
set -u
O=gpurun_out/s21
mkdir -p $O
: > $O/ab.jsonl
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?;
         echo "rc[$name]=$rc"; tail -1 $O/$name.log; [ $rc -eq 0 ] || exit $rc; }
rec() { echo "{\"arm\": \"$1\", \"bench\": $(grep -h '^{"metric"' $O/$1.log)}" >> $O/ab.jsonl; }
for i in 1 2; do
  step base_$i 300 python3 bench.py --gpus 1 --steps 10 --warmup 3; rec base_$i
  step wpi4_$i 300 env DLI_DECODE_WPI=4 python3 bench.py --gpus 1 --steps 10 --warmup 3; rec wpi4_$i
  step pipe_$i 300 env DLI_DECODE_PIPE=1 python3 bench.py --gpus 1 --steps 10 --warmup 3; rec pipe_$i
done
exit 0
