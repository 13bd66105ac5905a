#!/bin/bash
# Session 36 (round 6): Llama-3-70B bf16 on one GPU, 512 concurrent, on the final HEAD (round 5:
# 5,871 tok/s, profiles/r5/s28) — the same command as round 5.
set -u
O=gpurun_out/r6s36
mkdir -p $O
: > $O/bench.jsonl
timeout -k 10 700 python3 -u bench.py --model llama3-70b --steps 1 --warmup 1 --batch 512 > $O/llama70b_b512.log 2>&1
rc=$?; echo "rc[llama70b_b512]=$rc"; tail -2 $O/llama70b_b512.log | cut -c1-250; [ $rc -eq 0 ] || exit $rc
echo "{\"arm\": \"llama70b_b512\", \"bench\": $(grep -h '^{"metric"' $O/llama70b_b512.log)}" >> $O/bench.jsonl
exit 0
