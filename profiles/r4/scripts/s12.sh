#!/bin/bash
# round 4, session 12: default bench + rocprofv3 kernel summary (timed wave), pp2 same-GPU
# rehearsal over the default (IPC) data plane, Mixtral single vs ep4 same-GPU comparator
set -o pipefail
R=$(pwd); O=$R/gpurun_out/r4s12; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "rc[$name]=$rc"; tail -2 $O/$name.log | cut -c1-600; return $rc; }
step() { run "$@"; local rc=$?; [ $rc -le 1 ] || { echo "stop after rc=$rc"; exit $rc; }; }
step bench 400 python -u bench.py
step pp2 600 env DLI_DIST_BACKEND=gloo DLI_SAME_DEVICE=1 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 2
step mixtral_b256 600 python -u bench.py --model mixtral-8x7b --steps 2 --warmup 1 --batch 256
step ep4 700 env DLI_DIST_BACKEND=gloo DLI_SAME_DEVICE=1 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29543 bench.py --model mixtral-8x7b --gpus 4 --steps 2 --warmup 1 --batch 64
cd /tmp && export TMPDIR=/tmp
step prof 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 $R/bench.py --steps 1 --warmup 1
cd $R
python3 scripts/prof_summary.py $O/prof 40 > $O/prof_all.txt
python3 scripts/prof_summary.py $O/prof 40 --tail-ms 800 --gaps 10 > $O/prof_wave.txt
grep -c "Cijk_" $O/prof_all.txt > $O/cijk_count.txt || true
find $O/prof -name "*kernel_trace.csv" -exec gzip -1 {} \;
du -sh $O
echo "end $(date +%T)"
