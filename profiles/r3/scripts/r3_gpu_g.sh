# round 3, GPU session G: grid-split add+RMSNorm for batch 1..4, then the batch-1 bench and
# its rocprof kernel summary.
set -o pipefail
mkdir -p gpurun_out/r3g
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r3g
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "rc[$name]=$rc"; tail -4 $O/$name.log; return $rc; }
run kern 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "add_rmsnorm or gemv or fused" &&
run b1 300 python bench.py --steps 8 --warmup 1 --batch 1 &&
DLI_NORM_GRID=0 run b1_nogrid 300 python bench.py --steps 8 --warmup 1 --batch 1 &&
run b1_again 300 python bench.py --steps 8 --warmup 1 --batch 1 &&
run eng 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_engine_gpu.py &&
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null &&
run prof_b1 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_b1 -o b1 -- python bench.py --steps 2 --warmup 1 --batch 1 &&
python scripts/prof_summary.py $O/prof_b1 30 --tail-ms 500 --gaps 12 > $O/prof_b1_summary.txt; find $O/prof_b1 -name "*trace.csv" -delete
echo "end $(date +%T)"
