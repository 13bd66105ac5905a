#!/bin/bash
# Session 28: secondary configurations at round-5 HEAD (regression check against round 4):
# Llama-3-70B b512, Mixtral 8x7B b512, Llama-3-8B at 4 concurrent requests (the batch-1
# reduce-free chain at M = 4).
set -u
O=gpurun_out/s28
mkdir -p $O
: > $O/bench.jsonl
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?;
         echo "rc[$name]=$rc"; tail -2 $O/$name.log; [ $rc -eq 0 ] || exit $rc; }
rec() { echo "{\"arm\": \"$1\", \"bench\": $(grep -h '^{"metric"' $O/$1.log)}" >> $O/bench.jsonl; }
step b4 240 python3 bench.py --batch 4 --steps 4 --warmup 1
rec b4
step mixtral_b512 400 python3 -u bench.py --model mixtral-8x7b --steps 1 --warmup 1 --batch 512
rec mixtral_b512
step llama70b_b512 500 python3 -u bench.py --model llama3-70b --steps 1 --warmup 1 --batch 512
rec llama70b_b512
exit 0
