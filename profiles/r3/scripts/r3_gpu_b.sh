# round 3, GPU session B: IPC probe with captured (kernel) semaphores, PP-over-IPC GPU tests
# with the exchange captured in the decode graphs, pp2/pp4 same-GPU IPC benches + rocprof of
# pp2, slab-store A/B on the decode projections.
set -o pipefail
mkdir -p gpurun_out/r3b
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r3b
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "rc[$name]=$rc"; tail -3 $O/$name.log; return $rc; }
run probe 180 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29621 scripts/ipc_probe.py --flags device --out $O/probe.jsonl &&
run pp_ipc_tests 900 python -u -m pytest tests/test_parallel_gpu.py -x -v --timeout 300 --timeout-method thread &&
for st in 0 2 1; do run slab$st 600 python scripts/bench_decode_tiles.py --shapes down,o,qkv --slab-store $st --top 3 || exit 1; done &&
DLI_DIST_BACKEND=gloo DLI_SAME_DEVICE=1 DLI_PP_COMM=ipc run pp2_ipc 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29623 bench.py --gpus 2 --steps 2 --warmup 1 --batch 512 &&
DLI_DIST_BACKEND=gloo DLI_SAME_DEVICE=1 DLI_PP_COMM=ipc run pp4_ipc 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29624 bench.py --gpus 4 --steps 2 --warmup 1 --batch 256
echo "end $(date +%T)"
