#!/bin/bash
# Session 3 (round 6): the driver's 8-rank command form on one GPU without the per-rank
# autotune (8 ranks tuning one at a time on a shared GPU took > 15 min in s02), and the M = 512
# split-K slab-store probe (fp32 / bf16 / no partials).
set -u
O=gpurun_out/r6s03
mkdir -p $O
: > $O/bench.jsonl
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?;
         echo "rc[$name]=$rc"; tail -3 $O/$name.log; [ $rc -eq 0 ] || exit $rc; }
rec() { echo "{\"arm\": \"$1\", \"bench\": $(grep -h '^{"metric"' $O/$1.log)}" >> $O/bench.jsonl; }
step slab_probe 300 python3 -u scripts/slab_probe.py
step pp8_driver_form 800 env DLI_SAME_DEVICE=1 DLI_GEMM_AUTOTUNE=0 python3 -u bench.py --gpus 8 --steps 20 --warmup 5
rec pp8_driver_form
exit 0
