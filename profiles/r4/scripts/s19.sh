#!/bin/bash
# round 4, session 19: pruned library (4-wave tiles 34 / 41 / 45), Mixtral expert GEMMs:
# prefill-sized grouped GEMMs on the 8-phase vs the two-barrier 4-wave tile, decode b512 landscape
set -o pipefail
R=$(pwd); O=$R/gpurun_out/r4s19; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "rc[$name]=$rc"; tail -2 $O/$name.log | cut -c1-250; return $rc; }
step() { run "$@"; local rc=$?; [ $rc -le 1 ] || { echo "stop after rc=$rc"; exit $rc; }; }
step t4w 300 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "4wave or gemm"
step moe_prefill 400 python -u scripts/bench_moe_tiles.py --batch 16384 --tiles 22,45
step moe_b512 500 python -u scripts/bench_moe_tiles.py --batch 512
echo "end $(date +%T)"
