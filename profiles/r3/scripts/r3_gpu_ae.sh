#!/bin/bash
# batch-1: GEMV + add + RMSNorm in one kernel (last-workgroup reduce) vs the two-kernel path;
# batch-512: prefill GEMM autotune (8-phase vs hipBLASLt) vs 8-phase only
set -o pipefail
mkdir -p gpurun_out/r3ae
run() { local n=$1 t=$2; shift 2; echo "=== $n $(date +%T)"; timeout -k 10 $t "$@" > gpurun_out/r3ae/$n.log 2>&1; local rc=$?; echo "rc[$n]=$rc"; tail -2 gpurun_out/r3ae/$n.log | cut -c1-300; return $rc; }
run kern 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "gemv or splitk_add_rmsnorm" &&
run sweep_norm 300 python -u scripts/gemv_sweep.py --out gpurun_out/r3ae/sweep_norm.jsonl &&
DLI_GEMV_NORM=0 run sweep_nonorm 300 python -u scripts/gemv_sweep.py --out gpurun_out/r3ae/sweep_nonorm.jsonl &&
DLI_GEMM_AUTOTUNE_LOG=1 run b1_norm1 300 python -u bench.py --steps 16 --warmup 2 --batch 1 &&
DLI_GEMV_NORM=0 run b1_off1 300 python -u bench.py --steps 16 --warmup 2 --batch 1 &&
run b1_norm2 300 python -u bench.py --steps 16 --warmup 2 --batch 1 &&
DLI_GEMV_NORM=0 run b1_off2 300 python -u bench.py --steps 16 --warmup 2 --batch 1 &&
DLI_GEMM_AUTOTUNE_LOG=1 run b512_tp1 400 python -u bench.py --steps 4 --warmup 1 &&
DLI_TUNE_PREFILL=0 run b512_own1 400 python -u bench.py --steps 4 --warmup 1 &&
run b512_tp2 400 python -u bench.py --steps 4 --warmup 1 &&
DLI_TUNE_PREFILL=0 run b512_own2 400 python -u bench.py --steps 4 --warmup 1
echo "end $(date +%T)"
