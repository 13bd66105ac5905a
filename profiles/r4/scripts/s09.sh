#!/bin/bash
# round 4, session 09: RS GEMM tests + A/B, IPC endpoint test, bench A/Bs, pp2 rehearsal
set -o pipefail
O=gpurun_out/r4s09; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "rc[$name]=$rc"; tail -2 $O/$name.log | cut -c1-900; return $rc; }
run t4w 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "4wave"
run gemm_sq 300 python -u scripts/bench_gemm8p.py --only sq --tiles 22,41,43,44 --out $O/gemm_sq.json
run gemm_prefill 400 python -u scripts/bench_gemm8p.py --only prefill --tiles 22,41,43,44 --out $O/gemm_prefill.json
run gemm_decode 300 python -u scripts/bench_gemm8p.py --only b512 --tiles 22,41,43,44 --out $O/gemm_decode.json
run ipc_tests 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_ipc_gpu.py
run bench_default 400 python -u bench.py
run bench_noblas 400 env DLI_GEMM_NO_BLAS=1 python -u bench.py
echo "end $(date +%T)"
