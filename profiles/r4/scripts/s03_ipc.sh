#!/bin/bash
# round 4, session 03: hardened IPC data plane (uncached, sequenced, sticky, auto default),
# GEMM 4-wave diagnostics, pp2 same-GPU rehearsal vs single engine
set -o pipefail
O=gpurun_out/r4s03; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "rc[$name]=$rc"; tail -4 $O/$name.log | cut -c1-600; return $rc; }
run ipc_tests 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_ipc_gpu.py
run par_tests 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_parallel_gpu.py
run gemm_diag 300 python -u scripts/bench_gemm8p.py --only sq8192 --tiles 22,34,38,39 --out $O/gemm_diag.json
run gemm_diag2 300 python -u scripts/bench_gemm8p.py --only prefill_qkv --tiles 22,34,38,39 --out $O/gemm_diag2.json
run pp2 600 env DLI_DIST_BACKEND=gloo DLI_SAME_DEVICE=1 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 2 --warmup 1 --batch 256
run single256 400 python -u bench.py --steps 2 --warmup 1 --batch 256
echo "end $(date +%T)"
