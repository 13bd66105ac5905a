# round 3, session R: transposed-accumulator GEMMs in the engine: kernel + engine GPU tests,
# bench x2, b512 rocprof wave summary
set -o pipefail
mkdir -p gpurun_out/r3r
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r3r
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "rc[$name]=$rc"; tail -1 $O/$name.log | cut -c1-300; return $rc; }
run kern 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py &&
run eng 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_engine_gpu.py tests/test_hf_import.py &&
DLI_GEMM_AUTOTUNE_LOG=1 run b512_a 400 python -u bench.py --steps 5 --warmup 1 &&
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null &&
run prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o b512 -- python bench.py --steps 2 --warmup 1 &&
python scripts/prof_summary.py $O/prof 40 --tail-ms 900 --gaps 12 > $O/prof_summary.txt && find $O/prof -name "*trace.csv" -delete
echo "end $(date +%T)"
