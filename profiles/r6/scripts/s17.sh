#!/bin/bash
# Session 17 (round 6): the fused MoE gate (moe_router_kernel: logits + softmax + top-2 in
# one wave per token, replacing the 512 x 8 router GEMM, its split-K reduce and the route
# kernel) — kernel / engine / expert-parallel GPU tests, then a same-box Mixtral b512 A/B
# against the GEMM + route path.
set -u
O=gpurun_out/r6s17
mkdir -p $O
: > $O/bench.jsonl
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?;
         echo "rc[$name]=$rc"; tail -2 $O/$name.log; [ $rc -eq 0 ] || exit $rc; }
rec() { echo "{\"arm\": \"$1\", \"bench\": $(grep -h '^{"metric"' $O/$1.log)}" >> $O/bench.jsonl; }
PT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
step tests 600 $PT tests/test_kernels_gpu.py tests/test_engine_gpu.py tests/test_parallel_gpu.py -k "moe or router or mixtral or expert"
step fused_1 500 python3 -u bench.py --model mixtral-8x7b --steps 2 --warmup 1
rec fused_1
step gemm_1 500 env DLI_MOE_ROUTER_GEMM=1 python3 -u bench.py --model mixtral-8x7b --steps 2 --warmup 1
rec gemm_1
step fused_2 500 python3 -u bench.py --model mixtral-8x7b --steps 2 --warmup 1
rec fused_2
step gemm_2 500 env DLI_MOE_ROUTER_GEMM=1 python3 -u bench.py --model mixtral-8x7b --steps 2 --warmup 1
rec gemm_2
exit 0
