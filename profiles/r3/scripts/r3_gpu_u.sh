# round 3, session U: end-to-end config 2 with the faster control plane (aiohttp fronts,
# on-loop dispatcher, inline store) vs uvicorn fronts of the same code, and engine-only bench
set -o pipefail
mkdir -p gpurun_out/r3u
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r3u
e2e() { local name=$1 srv=$2; echo "=== e2e $name $(date +%T)"; timeout -k 10 560 bash scripts/serve_e2e.sh 4096 1024 512 $srv > $O/e2e_$name.log 2>&1; local rc=$?; mkdir -p $O/$name; mv gpurun_out/e2e_*.json $O/$name/ 2>/dev/null; echo "rc[$name]=$rc"; cat $O/$name/e2e_loadgen_c1024.json 2>/dev/null | cut -c1-250; return $rc; }
e2e aiohttp aiohttp &&
e2e uvicorn uvicorn &&
echo "=== bench $(date +%T)" && timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 > $O/bench.log 2>&1; echo "rc[bench]=$?"; tail -1 $O/bench.log | cut -c1-200
echo "end $(date +%T)"
