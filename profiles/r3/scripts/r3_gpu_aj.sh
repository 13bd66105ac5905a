#!/bin/bash
# round 3, session AJ: decode GEMMs — hipBLASLt as an extra autotune candidate (A/B)
set -o pipefail
mkdir -p gpurun_out/r3aj
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r3aj
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "rc[$name]=$rc"; tail -2 $O/$name.log | cut -c1-300; return $rc; }
run own1 400 python -u bench.py --steps 4 --warmup 1 &&
DLI_GEMM_DECODE_BLAS=1 DLI_GEMM_AUTOTUNE_LOG=1 run blas1 400 python -u bench.py --steps 4 --warmup 1 &&
run own2 400 python -u bench.py --steps 4 --warmup 1 &&
DLI_GEMM_DECODE_BLAS=1 run blas2 400 python -u bench.py --steps 4 --warmup 1
echo "end $(date +%T)"
