#!/bin/bash
# Session 7 (round 6): BASELINE config 4 in the driver's 8-rank form on one GPU — Llama-3-70B
# layer-sharded over 8 pipeline ranks (random init, then the reference flow: shard-model
# --num_shards 8 export -> every rank loads its own shard file via --shard-dir).
set -u
O=gpurun_out/r6s07
mkdir -p $O
: > $O/bench.jsonl
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?;
         echo "rc[$name]=$rc"; tail -2 $O/$name.log; [ $rc -eq 0 ] || exit $rc; }
rec() { echo "{\"arm\": \"$1\", \"bench\": $(grep -h '^{"metric"' $O/$1.log)}" >> $O/bench.jsonl; }
# (s06: the rocprofv3 wave of the fp16-slab default, then 70B pp8 ran out of HBM: every rank
# sized its KV pool before any weights were resident; fixed by counting pending weights)
export DLI_SAME_DEVICE=1 DLI_GEMM_AUTOTUNE=0
step llama70b_pp8 600 python3 -u bench.py --model llama3-70b --gpus 8 --batch 64 --steps 2 --warmup 1
rec llama70b_pp8
SH=${TMPDIR:-/tmp}/dli_r6_shards
df -h ${TMPDIR:-/tmp} | tee $O/df.txt
avail=$(df -Pk ${TMPDIR:-/tmp} | awk 'NR==2 {print $4}')
if [ "$avail" -lt 180000000 ]; then echo "not enough disk for the 141 GB export ($avail KiB)"; exit 0; fi
step export70b 700 python3 -u -m distributed_llm_inferencing_amd.cli shard-model --model_name llama3-70b --num_shards 8 --output_dir $SH
du -sh $SH | tee $O/du.txt
step llama70b_pp8_shards 700 python3 -u bench.py --model llama3-70b --gpus 8 --batch 64 --steps 2 --warmup 1 --shard-dir $SH/llama3-70b
rec llama70b_pp8_shards
rm -rf $SH
exit 0
