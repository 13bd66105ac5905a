#!/bin/bash
# round 4, session 01: baseline at round start (gpu tests, bench, prefill GEMM A/B)
set -o pipefail
O=gpurun_out/r4s01; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "rc[$name]=$rc"; tail -3 $O/$name.log | cut -c1-400; return $rc; }
run gemm8p 400 python -u scripts/bench_gemm8p.py --only prefill --tiles 22 --out $O/gemm8p.json &&
run gemm8p_sq 300 python -u scripts/bench_gemm8p.py --only sq8192 --tiles 22 --out $O/gemm8p_sq.json &&
run bench 400 python -u bench.py &&
run bench_noblas 400 env DLI_GEMM_NO_BLAS=1 python -u bench.py
echo "end $(date +%T)"
