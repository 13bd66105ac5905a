#!/bin/bash
# round 4, session 05: IPC tests (relaxed padded sizes), parallel GPU tests at defaults,
# GEMM 4-wave variants: interleaved DMA (34), burst (40), deep W ring (41/42), diagnostics 38/39
set -o pipefail
O=gpurun_out/r4s05; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "rc[$name]=$rc"; tail -4 $O/$name.log | cut -c1-700; return $rc; }
run t4w 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "4wave"
run gemm_sq 300 python -u scripts/bench_gemm8p.py --only sq8192 --tiles 22,34,40,41,38,39 --out $O/gemm_sq.json
run gemm_prefill 400 python -u scripts/bench_gemm8p.py --only prefill --tiles 22,34,41 --out $O/gemm_prefill.json
run gemm_decode 300 python -u scripts/bench_gemm8p.py --only b512 --tiles 22,34,41,42 --out $O/gemm_decode.json
run ipc_tests 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_ipc_gpu.py
run par_tests 700 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_parallel_gpu.py
echo "end $(date +%T)"
