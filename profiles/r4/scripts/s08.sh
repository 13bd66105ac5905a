#!/bin/bash
# round 4, session 08: register-staged 4-wave GEMM (43/44) vs LDS-DMA (34/41) vs 22 / hipBLASLt
set -o pipefail
O=gpurun_out/r4s08; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "rc[$name]=$rc"; tail -2 $O/$name.log | cut -c1-900; return $rc; }
run t4w 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "4wave"
run gemm_sq 300 python -u scripts/bench_gemm8p.py --only sq --tiles 22,34,41,43,44 --out $O/gemm_sq.json
run gemm_prefill 400 python -u scripts/bench_gemm8p.py --only prefill --tiles 22,41,43,44 --out $O/gemm_prefill.json
run gemm_decode 300 python -u scripts/bench_gemm8p.py --only b512 --tiles 22,41,43,44 --out $O/gemm_decode.json
echo "end $(date +%T)"
