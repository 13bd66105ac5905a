#!/bin/bash
# round 4, session 20: MoE prefill grouped GEMMs on tile 45 — GPU tests, Mixtral b512 bench
# (single engine) A/B against the 8-phase prefill tile
set -o pipefail
R=$(pwd); O=$R/gpurun_out/r4s20; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "rc[$name]=$rc"; grep -h '"value"' $O/$name.log | cut -c1-200; tail -1 $O/$name.log | cut -c1-200; return $rc; }
step() { run "$@"; local rc=$?; [ $rc -le 1 ] || { echo "stop after rc=$rc"; exit $rc; }; }
step moe_tests 300 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "moe"
step mixtral_b512 600 python -u bench.py --model mixtral-8x7b --steps 2 --warmup 1 --batch 512
step mixtral_b512_t22 600 env DLI_MOE_PREFILL_TILE=22 python -u bench.py --model mixtral-8x7b --steps 2 --warmup 1 --batch 512
step mixtral_b512_again 600 python -u bench.py --model mixtral-8x7b --steps 2 --warmup 1 --batch 512
echo "end $(date +%T)"
