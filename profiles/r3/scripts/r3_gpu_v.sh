# round 3, session V: end-to-end config 2 with mixed-step GEMM plans (8-phase heuristic for
# 512 < M, autotuned 640..1024 buckets when serving) — tuned vs heuristic-only, refill 30 ms
set -o pipefail
mkdir -p gpurun_out/r3v
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r3v
e2e() { local name=$1; shift; echo "=== e2e $name $(date +%T)"; env "$@" timeout -k 10 500 bash scripts/serve_e2e.sh 4096 1024 512 aiohttp > $O/e2e_$name.log 2>&1; local rc=$?; mkdir -p $O/$name; mv gpurun_out/e2e_*.json $O/$name/ 2>/dev/null; echo "rc[$name]=$rc"; cut -c1-200 $O/$name/e2e_loadgen_c1024.json 2>/dev/null; return $rc; }
e2e tuned DLI_TUNE_MIXED=1 &&
e2e heur DLI_TUNE_MIXED=0 &&
e2e tuned_r30 DLI_TUNE_MIXED=1 DLI_REFILL_INTERVAL_S=0.03
echo "end $(date +%T)"
