# round 3, GPU session A: IPC transport probes (copy kernel vs memcpy, device abort), PP over
# IPC GPU tests, single-engine bench, same-GPU pp2 bench over IPC vs gloo.
set -o pipefail
mkdir -p gpurun_out/r3a
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r3a
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "rc[$name]=$rc"; tail -4 $O/$name.log; return $rc; }
run probe_kernel 180 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29611 scripts/ipc_probe.py --flags device --out $O/probe_kernel.jsonl &&
DLI_IPC_COPY=memcpy run probe_memcpy 180 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29612 scripts/ipc_probe.py --flags device --out $O/probe_memcpy.jsonl &&
run pp_ipc_tests 600 python -u -m pytest tests/test_parallel_gpu.py -x -v --timeout 300 --timeout-method thread &&
run bench1 600 python bench.py --steps 3 --warmup 1 &&
DLI_DIST_BACKEND=gloo DLI_SAME_DEVICE=1 DLI_PP_COMM=ipc run pp2_ipc 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29613 bench.py --gpus 2 --steps 2 --warmup 1 --batch 512
echo "end $(date +%T)"
