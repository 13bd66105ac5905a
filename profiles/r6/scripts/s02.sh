#!/bin/bash
# Session 2 (round 6): the driver's exact 8-rank command form (pp8, --steps 20 --warmup 5) on
# one GPU, every rank on cuda:0 (IPC mailboxes), with the head's host time per tick.
set -u
O=gpurun_out/r6s02
mkdir -p $O
: > $O/bench.jsonl
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?;
         echo "rc[$name]=$rc"; tail -3 $O/$name.log; [ $rc -eq 0 ] || exit $rc; }
rec() { echo "{\"arm\": \"$1\", \"bench\": $(grep -h '^{"metric"' $O/$1.log)}" >> $O/bench.jsonl; }
step pp8_driver_form 1000 env DLI_SAME_DEVICE=1 python3 -u bench.py --gpus 8 --steps 20 --warmup 5
rec pp8_driver_form
exit 0
