#!/bin/bash
# Session 14 (round 6): decode attention at batch 512 against context length — the fused
# kernel with and without its V rows requested one tile ahead, and the unfused plain /
# pipelined kernels — to split its per-token streaming cost from its fixed cost.
set -u
O=gpurun_out/r6s14
mkdir -p $O
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?;
         echo "rc[$name]=$rc"; tail -8 $O/$name.log; [ $rc -eq 0 ] || exit $rc; }
step probe 300 python3 -u scripts/attn_probe.py --batch 64,512 --ctx 1,33,66,100,200
exit 0
