#!/bin/bash
# round 3, session AO: decode QKV plans timed with the attention path they feed (fused
# kernel or RoPE/cache + attention) vs with the RoPE/cache kernel only (A/B, batch 1 and 512)
set -o pipefail
mkdir -p gpurun_out/r3ao
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r3ao
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "rc[$name]=$rc"; tail -2 $O/$name.log | cut -c1-300; return $rc; }
run kern 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "attention or gemv or splitk" &&
DLI_GEMM_AUTOTUNE_LOG=1 run b1_new1 300 python -u bench.py --steps 16 --warmup 2 --batch 1 &&
DLI_TUNE_QKV_ATTN=0 DLI_GEMM_AUTOTUNE_LOG=1 run b1_old1 300 python -u bench.py --steps 16 --warmup 2 --batch 1 &&
run b1_new2 300 python -u bench.py --steps 16 --warmup 2 --batch 1 &&
DLI_TUNE_QKV_ATTN=0 run b1_old2 300 python -u bench.py --steps 16 --warmup 2 --batch 1 &&
DLI_GEMM_AUTOTUNE_LOG=1 run b512_new 400 python -u bench.py --steps 4 --warmup 1 &&
DLI_TUNE_QKV_ATTN=0 run b512_old 400 python -u bench.py --steps 4 --warmup 1
echo "end $(date +%T)"
