# round 3, GPU session C: full GPU test tier, N=1 bench, same-GPU pp2/pp4 benches over the IPC
# data plane with the exchange captured in the stage graphs, rocprof of the pp2 rehearsal.
set -o pipefail
mkdir -p gpurun_out/r3c
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r3c
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "rc[$name]=$rc"; tail -3 $O/$name.log; return $rc; }
run gputests 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread ; 
run bench1 600 python bench.py --steps 3 --warmup 1 &&
run bench_b1 600 python bench.py --steps 16 --warmup 2 --batch 1 &&
DLI_DIST_BACKEND=gloo DLI_SAME_DEVICE=1 DLI_PP_COMM=ipc run pp2_ipc 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29633 bench.py --gpus 2 --steps 2 --warmup 1 --batch 512 &&
DLI_DIST_BACKEND=gloo DLI_SAME_DEVICE=1 DLI_EP_COMM=ipc run ep4_ipc 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29636 bench.py --model mixtral-8x7b --gpus 4 --steps 1 --warmup 1 --batch 64 &&
DLI_DIST_BACKEND=gloo DLI_SAME_DEVICE=1 DLI_PP_COMM=ipc run pp4_ipc 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29634 bench.py --gpus 4 --steps 2 --warmup 1 --batch 256 &&
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null &&
DLI_DIST_BACKEND=gloo DLI_SAME_DEVICE=1 DLI_PP_COMM=ipc run prof_pp2 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29635 --no-python rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_pp2 -o pp2_%pid% -- python bench.py --gpus 2 --steps 1 --warmup 1 --batch 512 &&
python scripts/prof_summary.py $O/prof_pp2 30 --merge --tail-ms 2500 --gaps 12 > $O/prof_pp2_summary.txt; find $O/prof_pp2 -name "*trace.csv" -delete
echo "end $(date +%T)"
