# round 3, session AN: e2e config 2 at HEAD (prefill autotune, two-phase sampler)
# (16,384 requests at concurrency 1024) with the per-step trace, and bench.py on the same box
set -o pipefail
mkdir -p gpurun_out/r3an
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r3an
echo "=== bench $(date +%T)"; timeout -k 10 400 python -u bench.py --steps 5 --warmup 1 > $O/bench.log 2>&1; echo "rc[bench]=$?"; tail -1 $O/bench.log | cut -c1-160
echo "=== e2e $(date +%T)"; DLI_STEP_TRACE=$PWD/$O/steps.txt timeout -k 10 700 bash scripts/serve_e2e.sh 16384 1024 512 aiohttp > $O/e2e.log 2>&1; echo "rc[e2e]=$?"; mkdir -p $O/e2e; mv gpurun_out/e2e_*.json $O/e2e/ 2>/dev/null; cut -c1-220 $O/e2e/e2e_loadgen_c1024.json
echo "end $(date +%T)"
