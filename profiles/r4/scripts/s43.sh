#!/bin/bash
# round 4, session 43: config 2 end to end at HEAD (4,096 requests at concurrency 1024, then a
# lone request through every hop) after the batch-1 gate/up change
set -o pipefail
R=$(pwd); O=$R/gpurun_out/r4s43; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 bash scripts/serve_e2e.sh 4096 1024 512 aiohttp > $O/e2e.log 2>&1
rc=$?; echo "rc[e2e]=$rc"
cp gpurun_out/e2e_*.json $O/ 2>/dev/null
tail -15 $O/e2e.log | cut -c1-250
echo "end $(date +%T)"
exit $rc
