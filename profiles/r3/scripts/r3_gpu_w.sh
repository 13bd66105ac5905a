# round 3, session W: end-to-end config 2, master/worker CPU and control-plane latency split;
# one master process vs 4 (serve-master --procs 4: one port, one database, peer fan-out)
set -o pipefail
mkdir -p gpurun_out/r3w
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r3w
e2e() { local name=$1; shift; echo "=== e2e $name $(date +%T)"; env "$@" timeout -k 10 500 bash scripts/serve_e2e.sh 4096 1024 512 aiohttp > $O/e2e_$name.log 2>&1; local rc=$?; mkdir -p $O/$name; mv gpurun_out/e2e_*.json $O/$name/ 2>/dev/null; echo "rc[$name]=$rc"; cut -c1-200 $O/$name/e2e_loadgen_c1024.json 2>/dev/null; cat $O/$name/e2e_cpu.json; return $rc; }
e2e p1 DLI_MASTER_PROCS=1 &&
e2e p4 DLI_MASTER_PROCS=4 &&
echo "=== bench $(date +%T)" && timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 > $O/bench.log 2>&1; echo "rc[bench]=$?"; tail -1 $O/bench.log | cut -c1-200
echo "end $(date +%T)"
