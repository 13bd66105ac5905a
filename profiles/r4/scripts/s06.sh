#!/bin/bash
# round 4, session 06: IPC endpoint test; bench A/B: defaults vs deep-W 4-wave tile 41 in the
# autotune candidates vs no hipBLASLt; pp2 same-GPU rehearsal (IPC default) vs single engine
set -o pipefail
O=gpurun_out/r4s06; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "rc[$name]=$rc"; tail -2 $O/$name.log | cut -c1-700; return $rc; }
run ipc_tests 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_ipc_gpu.py
run bench_default 400 python -u bench.py
run bench_t41 400 env DLI_GEMM_EXCLUDE=26,27,35,36,37,42 DLI_GEMM_AUTOTUNE_LOG=1 python -u bench.py
run bench_noblas 400 env DLI_GEMM_NO_BLAS=1 python -u bench.py
run bench_noblas_t41 400 env DLI_GEMM_NO_BLAS=1 DLI_GEMM_EXCLUDE=26,27,35,36,37,42 python -u bench.py
run pp2 500 env DLI_DIST_BACKEND=gloo DLI_SAME_DEVICE=1 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1
echo "end $(date +%T)"
