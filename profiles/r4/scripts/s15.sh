#!/bin/bash
# round 4, session 15: why four processes on one GPU run the EP rehearsal at ~40 % of the
# single engine: ep2 (2 x 128), ep4 with 1 / 2 hardware queues per process
set -o pipefail
R=$(pwd); O=$R/gpurun_out/r4s15; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "rc[$name]=$rc"; grep -h '"value"' $O/$name.log | cut -c1-260; return $rc; }
step() { run "$@"; local rc=$?; [ $rc -le 1 ] || { echo "stop after rc=$rc"; exit $rc; }; }
step t4w 300 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "4wave or gemm"
EPR="python -u -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
step ep2 700 env DLI_DIST_BACKEND=gloo DLI_SAME_DEVICE=1 $EPR --nproc-per-node 2 --master-port 29553 bench.py --model mixtral-8x7b --gpus 2 --steps 2 --warmup 1 --batch 128
step ep4_q1 700 env GPU_MAX_HW_QUEUES=1 DLI_DIST_BACKEND=gloo DLI_SAME_DEVICE=1 $EPR --nproc-per-node 4 --master-port 29555 bench.py --model mixtral-8x7b --gpus 4 --steps 2 --warmup 1 --batch 64
step ep4_q2 700 env GPU_MAX_HW_QUEUES=2 DLI_DIST_BACKEND=gloo DLI_SAME_DEVICE=1 $EPR --nproc-per-node 4 --master-port 29557 bench.py --model mixtral-8x7b --gpus 4 --steps 2 --warmup 1 --batch 64
echo "end $(date +%T)"
