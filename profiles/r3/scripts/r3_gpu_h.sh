# round 3, GPU session H: graph-timed GEMM autotune + workgroup-per-item decode attention on
# the unfused path; batch-1 bench twice (plan stability), its rocprof summary, and the
# default (headline) bench to check the graph-timed autotune at batch 512.
set -o pipefail
mkdir -p gpurun_out/r3h
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r3h
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "rc[$name]=$rc"; tail -3 $O/$name.log; return $rc; }
run kern 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "add_rmsnorm or decode_attention or fused" &&
DLI_GEMM_AUTOTUNE_LOG=1 run b1 300 python bench.py --steps 8 --warmup 1 --batch 1 &&
DLI_GEMM_AUTOTUNE_LOG=1 run b1_again 300 python bench.py --steps 8 --warmup 1 --batch 1 &&
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null &&
run prof_b1 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_b1 -o b1 -- python bench.py --steps 2 --warmup 1 --batch 1 &&
python scripts/prof_summary.py $O/prof_b1 30 --tail-ms 500 --gaps 12 > $O/prof_b1_summary.txt && find $O/prof_b1 -name "*trace.csv" -delete &&
DLI_GEMM_AUTOTUNE_LOG=1 run bdef 600 python bench.py --steps 3 --warmup 1
echo "end $(date +%T)"
