#!/bin/bash
# round 4, session 14: EP grouped-GEMM plan keyed on expected routed rows + same-device
# tuning lock: parallel GPU tests, Mixtral single b256 vs ep4 (4 x 64) on one box, pp2
set -o pipefail
R=$(pwd); O=$R/gpurun_out/r4s14; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "rc[$name]=$rc"; tail -2 $O/$name.log | cut -c1-400; return $rc; }
step() { run "$@"; local rc=$?; [ $rc -le 1 ] || { echo "stop after rc=$rc"; exit $rc; }; }
step par_tests 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_parallel_gpu.py
step mixtral_b256 600 python -u bench.py --model mixtral-8x7b --steps 2 --warmup 1 --batch 256
step ep4 800 env DLI_GEMM_AUTOTUNE_LOG=1 DLI_DIST_BACKEND=gloo DLI_SAME_DEVICE=1 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29549 bench.py --model mixtral-8x7b --gpus 4 --steps 2 --warmup 1 --batch 64
step pp2 600 env DLI_DIST_BACKEND=gloo DLI_SAME_DEVICE=1 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29551 bench.py --gpus 2
step bench 400 python -u bench.py
echo "end $(date +%T)"
