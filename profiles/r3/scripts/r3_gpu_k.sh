# round 3, GPU session K: fused decode attention for unsplit QKV plans + QKV autotune timed
# with its RoPE/cache consumer. Tests, batch-512 bench x2, batch 1, b512 rocprof summary.
set -o pipefail
mkdir -p gpurun_out/r3k
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r3k
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "rc[$name]=$rc"; tail -1 $O/$name.log | cut -c1-220; return $rc; }
run kern 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "fused or decode_attention" &&
run eng 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_engine_gpu.py &&
DLI_GEMM_AUTOTUNE_LOG=1 run b512_a 400 python -u bench.py --steps 5 --warmup 1 &&
run b512_b 400 python -u bench.py --steps 5 --warmup 1 &&
DLI_DECODE_WPI=4 run b512_wpi4 400 python -u bench.py --steps 5 --warmup 1 &&
DLI_GEMM_AUTOTUNE_LOG=1 run b1 300 python -u bench.py --steps 8 --warmup 1 --batch 1 &&
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null &&
run prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o b512 -- python bench.py --steps 2 --warmup 1 &&
python scripts/prof_summary.py $O/prof 40 --tail-ms 900 --gaps 12 > $O/prof_summary.txt && find $O/prof -name "*trace.csv" -delete
echo "end $(date +%T)"
