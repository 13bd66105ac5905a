#!/bin/bash
# Session 9 (round 6): the reference's sharded flow on the GPU — shard-model --num_shards 8
# export, then every pipeline rank loads its own shard_<r>/ file (C++ safetensors loader,
# vocab-parallel head rows read from the tail's file) via bench.py --shard-dir: Llama-3-8B
# (16 GB export on local disk), then Llama-3-70B (141 GB) in /dev/shm when it fits.
set -u
O=gpurun_out/r6s09
mkdir -p $O
: > $O/bench.jsonl
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?;
         echo "rc[$name]=$rc"; tail -2 $O/$name.log; [ $rc -eq 0 ] || exit $rc; }
rec() { echo "{\"arm\": \"$1\", \"bench\": $(grep -h '^{"metric"' $O/$1.log)}" >> $O/bench.jsonl; }
export DLI_SAME_DEVICE=1 DLI_GEMM_AUTOTUNE=0
SH=${TMPDIR:-/tmp}/dli_r6_shards8b
step export8b 400 python3 -u -m distributed_llm_inferencing_amd.cli shard-model --model_name llama3-8b --num_shards 8 --output_dir $SH
du -sh $SH | tee $O/du8b.txt
step llama8b_pp8_shards 400 python3 -u bench.py --gpus 8 --steps 2 --warmup 1 --shard-dir $SH/llama3-8b
rec llama8b_pp8_shards
rm -rf $SH
df -h /dev/shm | tee $O/df_shm.txt
avail=$(df -Pk /dev/shm | awk 'NR==2 {print $4}')
if [ "$avail" -lt 175000000 ]; then echo "/dev/shm too small for the 141 GB 70B export ($avail KiB)"; exit 0; fi
SH=/dev/shm/dli_r6_shards70b
trap 'rm -rf /dev/shm/dli_r6_shards70b' EXIT
step export70b 600 python3 -u -m distributed_llm_inferencing_amd.cli shard-model --model_name llama3-70b --num_shards 8 --output_dir $SH
step llama70b_pp8_shards 600 python3 -u bench.py --model llama3-70b --gpus 8 --batch 64 --steps 2 --warmup 1 --shard-dir $SH/llama3-70b
rec llama70b_pp8_shards
exit 0
