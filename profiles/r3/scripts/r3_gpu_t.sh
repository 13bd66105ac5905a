# round 3, session T: deep-pipeline small tiles (40-44: 5-6 LDS buffers). Numerics for every
# tile, decode-projection landscape, bench x2 (autotune log)
set -o pipefail
mkdir -p gpurun_out/r3t
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r3t
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "rc[$name]=$rc"; tail -1 $O/$name.log | cut -c1-300; return $rc; }
run kern 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "gemm or grouped or moe or linear or fused" &&
run tiles 400 python -u scripts/bench_decode_tiles.py --shapes o,qkv,down --top 8 &&
DLI_GEMM_AUTOTUNE_LOG=1 run b512_a 400 python -u bench.py --steps 5 --warmup 1 &&
run b512_b 400 python -u bench.py --steps 5 --warmup 1
echo "end $(date +%T)"
