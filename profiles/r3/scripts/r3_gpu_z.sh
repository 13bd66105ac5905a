# round 3, session Z: e2e config 2 with a per-step engine trace (kind, rows, decode rows,
# tokens, running, waiting)
set -o pipefail
mkdir -p gpurun_out/r3z
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r3z
echo "=== e2e $(date +%T)"; DLI_STEP_TRACE=$PWD/$O/steps.txt timeout -k 10 500 bash scripts/serve_e2e.sh 4096 1024 512 aiohttp > $O/e2e.log 2>&1; echo "rc[e2e]=$?"; mkdir -p $O/e2e; mv gpurun_out/e2e_*.json $O/e2e/ 2>/dev/null; cut -c1-200 $O/e2e/e2e_loadgen_c1024.json; wc -l $O/steps.txt
echo "end $(date +%T)"
# reduce kernel with 512 threads per row (A/B on the decode projections with their consumers)
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "rc[$name]=$rc"; tail -1 $O/$name.log | cut -c1-200; return $rc; }
run tiles256 300 python -u scripts/bench_decode_tiles.py --shapes o,down --top 3 &&
DLI_REDUCE_THREADS=512 run tiles512 300 python -u scripts/bench_decode_tiles.py --shapes o,down --top 3 &&
run tiles256b 300 python -u scripts/bench_decode_tiles.py --shapes o,down --top 3
