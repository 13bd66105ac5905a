#!/bin/bash
# round 4, session 02: 4-wave 256x256 GEMM (tiles 34-37): correctness, then A/B vs tile 22 and hipBLASLt
set -o pipefail
O=gpurun_out/r4s02; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "rc[$name]=$rc"; tail -3 $O/$name.log | cut -c1-600; return $rc; }
run t4w 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "4wave" &&
run gemm_prefill 600 python -u scripts/bench_gemm8p.py --only prefill --tiles 22,34,35,36,37 --out $O/gemm_prefill.json &&
run gemm_sq 300 python -u scripts/bench_gemm8p.py --only sq --tiles 22,34,35,36,37 --out $O/gemm_sq.json &&
run gemm_decode 300 python -u scripts/bench_gemm8p.py --only b512 --tiles 22,34,35,36,37 --out $O/gemm_decode.json &&
run tall 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_kernels_gpu.py -k "all_tiles"
echo "end $(date +%T)"
