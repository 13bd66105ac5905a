#!/bin/bash
# round 4, session 13: rocprofv3 kernel summaries (csv) — Llama-3-8B b512 head (hipBLASLt
# share), Mixtral b256 single engine vs ep4 same-GPU (IPC default), traces summarised then
# removed (gpurun_out must stay under 64 MiB)
set -o pipefail
R=$(pwd); O=$R/gpurun_out/r4s13; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "rc[$name]=$rc"; tail -2 $O/$name.log | cut -c1-400; return $rc; }
step() { run "$@"; local rc=$?; [ $rc -le 1 ] || { echo "stop after rc=$rc"; exit $rc; }; }
summ() { local d=$1 tail=$2; shift 2
  python3 $R/scripts/prof_summary.py $d 60 "$@" > $d.all.txt
  python3 $R/scripts/prof_summary.py $d 60 --tail-ms $tail --gaps 10 "$@" > $d.wave.txt
  find $d -name "*kernel_stats.csv" -exec cp {} $d.stats.csv \; ; rm -rf $d; }
cd /tmp && export TMPDIR=/tmp
step prof_llama 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/llama_b512 -o run -- python3 $R/bench.py --steps 1 --warmup 1
summ $O/llama_b512 800
step prof_mixtral 700 rocprofv3 --kernel-trace --stats --output-format csv -d $O/mixtral_b256 -o run -- python3 $R/bench.py --model mixtral-8x7b --steps 1 --warmup 1 --batch 256
summ $O/mixtral_b256 1700
cd $R
step prof_ep4 800 env DLI_DIST_BACKEND=gloo DLI_SAME_DEVICE=1 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29547 --no-python rocprofv3 --kernel-trace --stats --output-format csv -d $O/ep4 -o ep_%pid% -- python3 bench.py --model mixtral-8x7b --gpus 4 --steps 1 --warmup 1 --batch 64
summ $O/ep4 4000 --merge
du -sh $O
echo "end $(date +%T)"
