#!/bin/bash
# round 4, session 11: IPC tests (zombie-aware liveness), bench A/B of the GEMM defaults on
# one box, rocprofv3 kernel summary of the default bench (no hipBLASLt kernel expected)
set -o pipefail
R=$(pwd); O=$R/gpurun_out/r4s11; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "rc[$name]=$rc"; tail -2 $O/$name.log | cut -c1-700; return $rc; }
step() { run "$@"; local rc=$?; [ $rc -le 1 ] || { echo "stop after rc=$rc"; exit $rc; }; }
step ipc_tests 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_ipc_gpu.py
step bench_default 400 python -u bench.py
step bench_no41decode 400 env DLI_GEMM_EXCLUDE=26,27,35,36,37,41,42,43,44 python -u bench.py
step bench_blas 400 env DLI_TUNE_PREFILL_BLAS=1 python -u bench.py
step bench_default2 400 python -u bench.py
cd /tmp && export TMPDIR=/tmp
step prof 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $R/bench.py --steps 1 --warmup 1
echo "end $(date +%T)"
