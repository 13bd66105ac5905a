#!/bin/bash
# round 4, session 07: Mixtral — grouped GEMM tiles incl. the 4-wave kernels (autotune log),
# EP comparator: single engine at 256 vs ep4 (IPC default) at 4 x 64 on one GPU
set -o pipefail
O=gpurun_out/r4s07; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "rc[$name]=$rc"; tail -2 $O/$name.log | cut -c1-700; return $rc; }
run mixtral_b512 700 env DLI_GEMM_AUTOTUNE_LOG=1 python -u bench.py --model mixtral-8x7b --steps 1 --warmup 1 --batch 512
run mixtral_b256 600 python -u bench.py --model mixtral-8x7b --steps 1 --warmup 1 --batch 256
run ep4 700 env DLI_DIST_BACKEND=gloo DLI_SAME_DEVICE=1 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29539 bench.py --model mixtral-8x7b --gpus 4 --steps 1 --warmup 1 --batch 64
echo "end $(date +%T)"
