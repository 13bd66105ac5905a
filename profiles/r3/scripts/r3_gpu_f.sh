# round 3, GPU session F: workgroup-per-item fused decode attention at small batch, and
# Infinity-Cache weight prefetch from a side stream (microbench + batch-1 bench A/B).
set -o pipefail
mkdir -p gpurun_out/r3f
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r3f
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "rc[$name]=$rc"; tail -4 $O/$name.log; return $rc; }
run kern 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "fused_rope or gemv or decode" &&
run pf_micro 300 python scripts/bench_prefetch.py &&
run b1_base 300 python bench.py --steps 8 --warmup 1 --batch 1 &&
DLI_PREFETCH=o run b1_pf_o 300 python bench.py --steps 8 --warmup 1 --batch 1 &&
DLI_PREFETCH=o,qkv run b1_pf_oqkv 300 python bench.py --steps 8 --warmup 1 --batch 1 &&
DLI_PREFETCH=o,qkv run eng_pf 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_engine_gpu.py
echo "end $(date +%T)"
