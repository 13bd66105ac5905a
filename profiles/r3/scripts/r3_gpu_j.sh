# round 3, GPU session J: same-box A/B of the graph-timed vs eager-timed autotune at the
# batch-512 headline, then a rocprof kernel summary of the headline step.
set -o pipefail
mkdir -p gpurun_out/r3j
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r3j
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "rc[$name]=$rc"; tail -1 $O/$name.log | cut -c1-200; return $rc; }
DLI_GEMM_TUNE_GRAPH=0 run eager_a 400 python -u bench.py --steps 5 --warmup 1 &&
DLI_GEMM_TUNE_GRAPH=1 run graph_a 400 python -u bench.py --steps 5 --warmup 1 &&
DLI_GEMM_TUNE_GRAPH=0 run eager_b 400 python -u bench.py --steps 5 --warmup 1 &&
DLI_GEMM_TUNE_GRAPH=1 run graph_b 400 python -u bench.py --steps 5 --warmup 1 &&
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null &&
run prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o b512 -- python bench.py --steps 2 --warmup 1 &&
python scripts/prof_summary.py $O/prof 40 --tail-ms 900 --gaps 12 > $O/prof_summary.txt && find $O/prof -name "*trace.csv" -delete
echo "end $(date +%T)"
