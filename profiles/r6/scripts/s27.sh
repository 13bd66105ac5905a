#!/bin/bash
# Session 27 (round 6): the multi-rank forms on the final HEAD, every rank on one GPU — the
# driver's pp8 / pp2 commands, Llama-3-70B pp8, Mixtral ep4 and ep8 (the expert-parallel
# path with the gate computed in the O-projection's reduce).
set -u
O=gpurun_out/r6s27
mkdir -p $O
: > $O/bench.jsonl
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?;
         echo "rc[$name]=$rc"; tail -2 $O/$name.log; [ $rc -eq 0 ] || exit $rc; }
rec() { echo "{\"arm\": \"$1\", \"bench\": $(grep -h '^{"metric"' $O/$1.log)}" >> $O/bench.jsonl; }
export DLI_SAME_DEVICE=1 DLI_GEMM_AUTOTUNE=0
step pp8 400 python3 -u bench.py --gpus 8 --steps 3 --warmup 1
rec pp8
step pp2 300 python3 -u bench.py --gpus 2 --steps 3 --warmup 1
rec pp2
step mixtral_ep4 400 python3 -u bench.py --model mixtral-8x7b --gpus 4 --batch 64 --steps 2 --warmup 1
rec mixtral_ep4
step mixtral_ep8 600 python3 -u bench.py --model mixtral-8x7b --gpus 8 --steps 2 --warmup 1
rec mixtral_ep8
step llama70b_pp8 600 python3 -u bench.py --model llama3-70b --gpus 8 --batch 64 --steps 2 --warmup 1
rec llama70b_pp8
exit 0
