#!/bin/bash
# Session 4 (round 6): head host time per tick after the pinned sampling-parameter ring
# (pp8, same GPU), the pp2 / pp4 forms of the driver's scaling run, and Mixtral ep4 / ep8 on
# one GPU with the shared-memory lockstep board (lockstep host ms per step).
set -u
O=gpurun_out/r6s04
mkdir -p $O
: > $O/bench.jsonl
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?;
         echo "rc[$name]=$rc"; tail -2 $O/$name.log; [ $rc -eq 0 ] || exit $rc; }
rec() { echo "{\"arm\": \"$1\", \"bench\": $(grep -h '^{"metric"' $O/$1.log)}" >> $O/bench.jsonl; }
export DLI_SAME_DEVICE=1 DLI_GEMM_AUTOTUNE=0
step pp8 300 python3 -u bench.py --gpus 8 --steps 3 --warmup 1
rec pp8
step pp4 300 python3 -u bench.py --gpus 4 --steps 3 --warmup 1
rec pp4
step pp2 300 python3 -u bench.py --gpus 2 --steps 3 --warmup 1
rec pp2
step mixtral_ep4_gloo 400 env DLI_EP_CTRL=gloo python3 -u bench.py --model mixtral-8x7b --gpus 4 --batch 64 --steps 2 --warmup 1
rec mixtral_ep4_gloo
step mixtral_ep4_shm 400 python3 -u bench.py --model mixtral-8x7b --gpus 4 --batch 64 --steps 2 --warmup 1
rec mixtral_ep4_shm
step mixtral_ep8 600 python3 -u bench.py --model mixtral-8x7b --gpus 8 --steps 2 --warmup 1
rec mixtral_ep8
exit 0
