#!/bin/bash
# Session 1 (round 6): HEAD single-engine bench (A/B anchor for this round) and the first
# rehearsal of the driver's 8-rank pp form on one GPU (every rank on cuda:0, IPC mailboxes).
set -u
O=gpurun_out/r6s01
mkdir -p $O
: > $O/bench.jsonl
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?;
         echo "rc[$name]=$rc"; tail -3 $O/$name.log; [ $rc -eq 0 ] || exit $rc; }
rec() { echo "{\"arm\": \"$1\", \"bench\": $(grep -h '^{"metric"' $O/$1.log)}" >> $O/bench.jsonl; }
step single 240 python3 -u bench.py --steps 8 --warmup 2
rec single
step pp8_same 700 env DLI_SAME_DEVICE=1 DLI_GEMM_AUTOTUNE=0 python3 -u bench.py --gpus 8 --steps 2 --warmup 1
rec pp8_same
exit 0
