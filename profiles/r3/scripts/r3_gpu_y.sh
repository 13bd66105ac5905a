# round 3, session Y: full GPU tier + smoke + bench at HEAD, then one e2e arm with the
# scheduler's preemption / KV counters in the worker metrics
set -o pipefail
mkdir -p gpurun_out/r3y
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r3y
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "rc[$name]=$rc"; tail -2 $O/$name.log | cut -c1-300; return $rc; }
run pytest 1000 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread &&
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" &&
run bench 400 python -u bench.py --steps 5 --warmup 1 &&
echo "=== e2e $(date +%T)" && timeout -k 10 500 bash scripts/serve_e2e.sh 4096 1024 512 aiohttp > $O/e2e.log 2>&1; echo "rc[e2e]=$?"; mkdir -p $O/e2e; mv gpurun_out/e2e_*.json $O/e2e/ 2>/dev/null; cut -c1-200 $O/e2e/e2e_loadgen_c1024.json
echo "end $(date +%T)"
