#!/bin/bash
# Session 5 (round 6): fp16 split-K slabs (EPI "slab16") — kernel numerics, engine and pp8
# GPU tests (mixed steps on heuristic plans, run alone), then a same-box alternated bench A/B
# of fp16 vs fp32 slabs with a rocprofv3 wave of the new default.
set -u
O=gpurun_out/r6s05
mkdir -p $O
: > $O/bench.jsonl
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?;
         echo "rc[$name]=$rc"; tail -2 $O/$name.log; [ $rc -eq 0 ] || exit $rc; }
rec() { echo "{\"arm\": \"$1\", \"bench\": $(grep -h '^{"metric"' $O/$1.log)}" >> $O/bench.jsonl; }
PT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
step mixed_alone 300 $PT tests/test_engine_gpu.py::test_mixed_steps_token_identical_on_gpu
step kernels 600 $PT tests/test_kernels_gpu.py -k "fp16_slabs or splitk or fused_rope or rope_cache or decode_attention"
step pp8_test 500 $PT tests/test_parallel_gpu.py -k pp8
step engine 600 $PT tests/test_engine_gpu.py
step ab_s16_1 240 python3 -u bench.py --steps 8 --warmup 2
rec ab_s16_1
step ab_f32_1 240 env DLI_SLAB_FP32=1 python3 -u bench.py --steps 8 --warmup 2
rec ab_f32_1
step ab_s16_2 240 python3 -u bench.py --steps 8 --warmup 2
rec ab_s16_2
step ab_f32_2 240 env DLI_SLAB_FP32=1 python3 -u bench.py --steps 8 --warmup 2
rec ab_f32_2
exit 0
