# round 3, GPU session E: GEMV unroll-4 tile + fused (unsplit) attention at tiny batch.
# Numerics first, then per-candidate M = 1 timings, a batch-1 bench and its rocprof summary.
set -o pipefail
mkdir -p gpurun_out/r3e
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r3e
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "rc[$name]=$rc"; tail -3 $O/$name.log; return $rc; }
run kern 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_engine_gpu.py &&
run tiles_m1 600 python scripts/bench_decode_tiles.py --m 1 --shapes qkv,o,gate_up,down --top 6 &&
DLI_GEMM_AUTOTUNE_LOG=1 run b1_tune 600 python bench.py --steps 8 --warmup 1 --batch 1 &&
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null &&
run prof_b1 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_b1 -o b1 -- python bench.py --steps 2 --warmup 1 --batch 1 &&
python scripts/prof_summary.py $O/prof_b1 30 --tail-ms 500 --gaps 12 > $O/prof_b1_summary.txt; find $O/prof_b1 -name "*trace.csv" -delete
echo "end $(date +%T)"
