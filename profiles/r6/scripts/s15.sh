#!/bin/bash
# Session 15 (round 6): BASELINE.json config 2 end to end on the round-6 engine — master
# (aiohttp front, sqlite store, dispatcher) -> one Llama-3-8B worker over HTTP, 4,096
# requests at concurrency 1024, then 16 lone requests (scripts/serve_e2e.sh); then the
# engine-only bench on the same box for the ratio.
set -u
O=gpurun_out/r6s15${E2E_TAG:-}
mkdir -p $O
timeout -k 10 1000 bash scripts/serve_e2e.sh ${E2E_N:-4096} 1024 512 aiohttp > $O/e2e.log 2>&1
rc=$?; echo "rc[e2e]=$rc"; tail -5 $O/e2e.log
cp gpurun_out/e2e_loadgen_c1024.json gpurun_out/e2e_loadgen_c1.json gpurun_out/e2e_cpu.json gpurun_out/e2e_metrics_after.json $O/ 2>/dev/null
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1
rc=$?; echo "rc[bench]=$rc"; tail -1 $O/bench.log
exit $rc
