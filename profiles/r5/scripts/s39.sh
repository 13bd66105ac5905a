#!/bin/bash
# Session 39: the LM head with the 4-wave tiles admitted (DLI_GEMM_HEAD_4W=1: tiles 45 and
# the persistent 55 race tile 22 for the fp32 head), alternated with the default, 10 steps.
set -u
O=gpurun_out/s39
mkdir -p $O
: > $O/ab.jsonl
run() { local name=$1; shift; echo "== $name"; timeout -k 10 300 "$@" > $O/$name.log 2>&1; local rc=$?;
        echo "rc[$name]=$rc"; [ $rc -eq 0 ] || exit $rc;
        echo "{\"arm\": \"$name\", \"bench\": $(grep -h '^{"metric"' $O/$name.log)}" >> $O/ab.jsonl; }
for i in 1 2; do
  run base_$i python3 bench.py --gpus 1 --steps 10 --warmup 3
  run head4w_$i env DLI_GEMM_HEAD_4W=1 DLI_GEMM_AUTOTUNE_LOG=1 python3 bench.py --gpus 1 --steps 10 --warmup 3
done
grep "autotune\] M=512 N=128256" $O/head4w_1.log $O/head4w_2.log > $O/head_picks.txt || true
exit 0
