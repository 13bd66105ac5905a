#!/bin/bash
# Session 8 (round 6): Mixtral grouped down projection as fp16 split-K slabs reduced inside
# the combine — GPU tests, the decode-sized plan sweep (weight-streaming TB/s) and a Mixtral
# b512 A/B against fp32 slabs; plus Llama-3-8B with the 256x224 gate/up tile (26) admitted to
# the decode autotune (fills 256 CUs) against the default candidate list.
set -u
O=gpurun_out/r6s08
mkdir -p $O
: > $O/bench.jsonl
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?;
         echo "rc[$name]=$rc"; tail -2 $O/$name.log; [ $rc -eq 0 ] || exit $rc; }
rec() { echo "{\"arm\": \"$1\", \"bench\": $(grep -h '^{"metric"' $O/$1.log)}" >> $O/bench.jsonl; }
PT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
step tests 400 $PT tests/test_kernels_gpu.py -k "moe"
step moe_tiles 400 python3 -u scripts/bench_moe_tiles.py --which down,gate_up
step mixtral_s16 500 python3 -u bench.py --model mixtral-8x7b --steps 2 --warmup 1
rec mixtral_s16
step mixtral_f32 500 env DLI_SLAB_FP32=1 python3 -u bench.py --model mixtral-8x7b --steps 2 --warmup 1
rec mixtral_f32
step llama_t26 240 env DLI_GEMM_EXCLUDE=34,41,45,55 python3 -u bench.py --steps 8 --warmup 2
rec llama_t26
step llama_def 240 python3 -u bench.py --steps 8 --warmup 2
rec llama_def
exit 0
