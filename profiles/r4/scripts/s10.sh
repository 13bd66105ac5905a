#!/bin/bash
# round 4, session 10: branch-free GELU (no accumulator scratch in gemm4w), 4-wave tests with
# repeats, full kernel tests, IPC tests, bench with hipBLASLt off the default prefill path
set -o pipefail
O=gpurun_out/r4s10; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "rc[$name]=$rc"; tail -2 $O/$name.log | cut -c1-900; return $rc; }
# pytest exit 1 = a test failed (numerics): keep going; anything else (fault, abort, timeout) stops
step() { run "$@"; local rc=$?; [ $rc -le 1 ] || { echo "stop after rc=$rc"; exit $rc; }; }
step t4w 300 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "4wave"
step kernels 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py
step ipc_tests 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_ipc_gpu.py
step bench_default 400 python -u bench.py
echo "end $(date +%T)"
