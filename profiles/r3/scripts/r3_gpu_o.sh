# round 3, GPU session O: 256x128 ping-pong GEMM (tile 28). Numerics for every tile /
# grouped mode, Mixtral grouped-GEMM candidate timings, Mixtral b512 bench, Llama b512 bench.
set -o pipefail
mkdir -p gpurun_out/r3o
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r3o
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "rc[$name]=$rc"; tail -1 $O/$name.log | cut -c1-250; return $rc; }
run kern 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "gemm or grouped or moe" &&
run moe_tiles 400 python -u scripts/bench_moe_tiles.py --batch 512 --which down,gate_up &&
DLI_GEMM_AUTOTUNE_LOG=1 run mixtral 600 python -u bench.py --model mixtral-8x7b --steps 2 --warmup 1 &&
DLI_GEMM_AUTOTUNE_LOG=1 run llama 400 python -u bench.py --steps 5 --warmup 1 &&
DLI_GEMM_EXCLUDE=26,27,28 run llama_no28 400 python -u bench.py --steps 5 --warmup 1
echo "end $(date +%T)"
