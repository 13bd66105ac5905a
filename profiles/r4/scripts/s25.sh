#!/bin/bash
# round 4, session 25: the library's DMA addressing in the two-barrier 4-wave GEMM (47: a
# voffset VGPR per piece, soffset 0, per-K-tile descriptor base) vs 45; PMC pass for both
set -o pipefail
R=$(pwd); O=$R/gpurun_out/r4s25; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "rc[$name]=$rc"; tail -2 $O/$name.log | cut -c1-200; return $rc; }
step() { run "$@"; local rc=$?; [ $rc -le 1 ] || { echo "stop after rc=$rc"; exit $rc; }; }
step t4w 300 env DLI_TEST_4W_TILES=45,47 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "4wave"
step gemm_sq 400 python -u scripts/bench_gemm8p.py --only sq --tiles 22,45,47 --out $O/gemm_sq.json
step gemm_prefill 500 python -u scripts/bench_gemm8p.py --only prefill --tiles 22,45,47 --out $O/gemm_prefill.json
echo "end $(date +%T)"
