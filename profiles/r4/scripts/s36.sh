#!/bin/bash
# round 4, session 36: pp2 same-GPU rehearsal over the default (uncached, sequence-checked)
# IPC data plane under rocprofv3: both ranks' kernels merged — GPU busy, ipc kernel share
set -o pipefail
R=$(pwd); O=$R/gpurun_out/r4s36; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "rc[$name]=$rc"; grep -h '"value"' $O/$name.log | cut -c90-220; tail -1 $O/$name.log | cut -c1-200; return $rc; }
step() { run "$@"; local rc=$?; [ $rc -le 1 ] || { echo "stop after rc=$rc"; exit $rc; }; }
step prof_pp2 700 env DLI_DIST_BACKEND=gloo DLI_SAME_DEVICE=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29567 --no-python rocprofv3 --kernel-trace --stats --output-format csv -d $O/pp2 -o pp2_%pid% -- python3 bench.py --gpus 2 --steps 1 --warmup 1
python3 scripts/prof_summary.py $O/pp2 40 --merge --tail-ms 2300 --gaps 10 > $O/pp2.wave.txt
rm -rf $O/pp2
head -30 $O/pp2.wave.txt | cut -c1-150
echo "end $(date +%T)"
