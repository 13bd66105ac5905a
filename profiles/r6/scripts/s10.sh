#!/bin/bash
# Session 10 (round 6): the 128x128 ping-pong tile (60: tile 28's schedule at BM = 128) —
# every GEMM test that walks the tile list, the grouped / MoE tests, the decode-sized MoE plan
# sweep, Mixtral b512 and the Llama-3-8B headline (tile 60 joins its decode autotune too).
set -u
O=gpurun_out/r6s10
mkdir -p $O
: > $O/bench.jsonl
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?;
         echo "rc[$name]=$rc"; tail -2 $O/$name.log; [ $rc -eq 0 ] || exit $rc; }
rec() { echo "{\"arm\": \"$1\", \"bench\": $(grep -h '^{"metric"' $O/$1.log)}" >> $O/bench.jsonl; }
PT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
step tests 600 $PT tests/test_kernels_gpu.py -k "all_tiles or pingpong or grouped or moe or fp16_slabs"
step moe_tiles 400 python3 -u scripts/bench_moe_tiles.py --which down,gate_up
step mixtral_1 500 python3 -u bench.py --model mixtral-8x7b --steps 2 --warmup 1
rec mixtral_1
step llama_1 240 python3 -u bench.py --steps 8 --warmup 2
rec llama_1
step mixtral_2 500 python3 -u bench.py --model mixtral-8x7b --steps 2 --warmup 1
rec mixtral_2
exit 0
