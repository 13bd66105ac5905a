#!/bin/bash
# Session 26 (round 6): 160x256 / 160x192 generic tiles (62 / 63) for the Mixtral decode
# expert GEMMs — GEMM / grouped / MoE GPU tests over every tile, the decode-sized grouped
# plan sweep, and Mixtral b512 with them in the grouped autotune.
set -u
O=gpurun_out/r6s26
mkdir -p $O
: > $O/bench.jsonl
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?;
         echo "rc[$name]=$rc"; tail -2 $O/$name.log; [ $rc -eq 0 ] || exit $rc; }
rec() { echo "{\"arm\": \"$1\", \"bench\": $(grep -h '^{"metric"' $O/$1.log)}" >> $O/bench.jsonl; }
PT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
step tests 600 $PT tests/test_kernels_gpu.py -k "all_tiles or asymmetric or grouped or moe or permutation or strided"
step moe_tiles 500 python3 -u scripts/bench_moe_tiles.py --which gate_up,down
grep '^{' $O/moe_tiles.log | head -12
step mixtral_1 500 python3 -u bench.py --model mixtral-8x7b --steps 4 --warmup 1
rec mixtral_1
step mixtral_2 500 python3 -u bench.py --model mixtral-8x7b --steps 4 --warmup 1
rec mixtral_2
exit 0
