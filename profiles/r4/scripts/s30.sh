#!/bin/bash
# round 4, session 30: EP on the GPU after the prefill cap — parallel GPU tests (EP N=2/4 over
# IPC graphs, pipeline), ep2 same-GPU bench
set -o pipefail
R=$(pwd); O=$R/gpurun_out/r4s30; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "rc[$name]=$rc"; grep -h '"value"' $O/$name.log | cut -c90-220; tail -1 $O/$name.log | cut -c1-200; return $rc; }
step() { run "$@"; local rc=$?; [ $rc -le 1 ] || { echo "stop after rc=$rc"; exit $rc; }; }
step par_tests 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_parallel_gpu.py tests/test_ipc_gpu.py
step ep2 700 env DLI_DIST_BACKEND=gloo DLI_SAME_DEVICE=1 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29563 bench.py --model mixtral-8x7b --gpus 2 --steps 2 --warmup 1 --batch 128
echo "end $(date +%T)"
