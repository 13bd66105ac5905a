# round 3, session X: end-to-end config 2 with batch-shape diagnostics (decode rows, running /
# waiting per step); default pacing vs no pacing
set -o pipefail
mkdir -p gpurun_out/r3x
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r3x
e2e() { local name=$1; shift; echo "=== e2e $name $(date +%T)"; env "$@" timeout -k 10 500 bash scripts/serve_e2e.sh 4096 1024 512 aiohttp > $O/e2e_$name.log 2>&1; local rc=$?; mkdir -p $O/$name; mv gpurun_out/e2e_*.json $O/$name/ 2>/dev/null; echo "rc[$name]=$rc"; cut -c1-200 $O/$name/e2e_loadgen_c1024.json 2>/dev/null; return $rc; }
e2e base DLI_MASTER_PROCS=1 &&
e2e nopace DLI_MASTER_PROCS=1 DLI_REFILL_INTERVAL_S=0 DLI_ADMIT_WINDOW_S=0
echo "end $(date +%T)"
