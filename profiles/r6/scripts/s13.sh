#!/bin/bash
# Session 13 (round 6): the weight-stationary grouped tile (61: the 256x224 8-phase kernel
# with its operands swapped, 256 weight rows x 224 routed rows) for the Mixtral decode expert
# GEMMs — GPU tests over every tile path that touches it, the decode-sized plan sweep, and a
# same-box Mixtral b512 A/B with tile 61 kept out of the grouped autotune.
set -u
O=gpurun_out/r6s13
mkdir -p $O
: > $O/bench.jsonl
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?;
         echo "rc[$name]=$rc"; tail -2 $O/$name.log; [ $rc -eq 0 ] || exit $rc; }
rec() { echo "{\"arm\": \"$1\", \"bench\": $(grep -h '^{"metric"' $O/$1.log)}" >> $O/bench.jsonl; }
PT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
step tests 500 $PT tests/test_kernels_gpu.py -k "weight_stationary or grouped or moe or all_tiles or asymmetric or pingpong"
step moe_tiles 500 python3 -u scripts/bench_moe_tiles.py --which down,gate_up
step mixtral_61 500 python3 -u bench.py --model mixtral-8x7b --steps 2 --warmup 1
rec mixtral_61
step mixtral_no61 500 env DLI_GEMM_EXCLUDE=26,34,41,45,55,61 python3 -u bench.py --model mixtral-8x7b --steps 2 --warmup 1
rec mixtral_no61
step mixtral_61b 500 python3 -u bench.py --model mixtral-8x7b --steps 2 --warmup 1
rec mixtral_61b
exit 0
