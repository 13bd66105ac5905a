# round 3, session AD: GEMV tile 33 (32 rows, 4 K-steps in flight; SiLU gate/up at M = 1):
# numerics, batch-1 bench x2 with the autotune log
set -o pipefail
mkdir -p gpurun_out/r3ad
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r3ad
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "rc[$name]=$rc"; tail -1 $O/$name.log | cut -c1-260; return $rc; }
run kern 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "gemv or gemm_bf16_all" &&
DLI_GEMM_AUTOTUNE_LOG=1 run b1a 300 python -u bench.py --steps 16 --warmup 2 --batch 1 &&
run b1b 300 python -u bench.py --steps 16 --warmup 2 --batch 1 &&
DLI_GEMM_EXCLUDE=26,27,33 run b1_no33 300 python -u bench.py --steps 16 --warmup 2 --batch 1
echo "end $(date +%T)"
# prefill plain GEMMs (QKV / O / down, no fused epilogue) on hipBLASLt vs tile 22
run b512_own1 400 python -u bench.py --steps 4 --warmup 1 &&
DLI_GEMM_PREFILL_BLAS=1 run b512_blas1 400 python -u bench.py --steps 4 --warmup 1 &&
run b512_own2 400 python -u bench.py --steps 4 --warmup 1 &&
DLI_GEMM_PREFILL_BLAS=1 run b512_blas2 400 python -u bench.py --steps 4 --warmup 1
echo "end $(date +%T)"
