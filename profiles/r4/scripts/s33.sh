#!/bin/bash
# round 4, session 33: config 2 end to end at HEAD with 16,384 requests (the round-3 e2e
# comparison), the single-engine bench on the same box, and pp4 same-GPU at 512 per microbatch
set -o pipefail
R=$(pwd); O=$R/gpurun_out/r4s33; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "rc[$name]=$rc"; grep -h '"value"\|"requests_per_s"' $O/$name.log | cut -c1-220; return $rc; }
step() { run "$@"; local rc=$?; [ $rc -le 1 ] || { echo "stop after rc=$rc"; exit $rc; }; }
step bench 400 python -u bench.py --steps 5 --warmup 2
step e2e 900 bash scripts/serve_e2e.sh 16384 1024 512 aiohttp
cp gpurun_out/e2e_*.json $O/ 2>/dev/null
step pp4_b512 800 env DLI_DIST_BACKEND=gloo DLI_SAME_DEVICE=1 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29565 bench.py --gpus 4 --steps 2 --warmup 1
echo "end $(date +%T)"
