#!/bin/bash
# round 4, session 28: refresh the secondary configs at HEAD — Llama-3-70B b512 (one GPU),
# pp4 same-GPU rehearsal at 256 per microbatch (default IPC data plane), Mixtral b128
set -o pipefail
R=$(pwd); O=$R/gpurun_out/r4s28; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "rc[$name]=$rc"; grep -h '"value"' $O/$name.log | cut -c90-260; tail -1 $O/$name.log | cut -c1-150; return $rc; }
step() { run "$@"; local rc=$?; [ $rc -le 1 ] || { echo "stop after rc=$rc"; exit $rc; }; }
step llama70b_b512 900 python -u bench.py --model llama3-70b --steps 1 --warmup 1 --batch 512
step pp4_b256 700 env DLI_DIST_BACKEND=gloo DLI_SAME_DEVICE=1 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 4 --batch 256 --steps 2 --warmup 1
step single_b256 400 python -u bench.py --batch 256
step mixtral_b128 600 python -u bench.py --model mixtral-8x7b --steps 2 --warmup 1 --batch 128
echo "end $(date +%T)"
