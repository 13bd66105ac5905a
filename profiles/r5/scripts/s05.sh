#!/bin/bash
# Session 5: GPU kernel/engine/parallel tests, then a same-box A/B of decode-step knobs on the driver's bench (alternated x2):
# sc1 (write-through) split-K slab stores for the generic-tile family (decode O / QKV), and
# the 256x224 gate/up tile admitted to the autotune; then a rocprofv3 wave summary at HEAD
# (summarised on the box: the raw trace exceeds what gpurun copies back).
set -u
O=gpurun_out/s05
mkdir -p $O
: > $O/ab.jsonl
run() { local arm=$1 r=$2; shift 2; timeout -k 10 240 env "$@" python3 bench.py --gpus 1 --steps 10 --warmup 3 > $O/${arm}_$r.log 2>&1;
        local rc=$?; echo "rc[$arm $r]=$rc"; [ $rc -eq 0 ] || { tail -20 $O/${arm}_$r.log; exit $rc; }
        echo "{\"arm\": \"$arm\", \"run\": $r, \"bench\": $(grep -h '^{"metric"' $O/${arm}_$r.log)}" >> $O/ab.jsonl
        grep -o '"value": [0-9.]*' $O/${arm}_$r.log; }
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_engine_gpu.py tests/test_parallel_gpu.py -k "not batch_invariant" > $O/tests.log 2>&1
rc=$?; echo "rc[tests]=$rc"; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  run base $r DLI_AB=0
  run fp32_logits $r DLI_FP32_LOGITS=1
  run tiles_sc1 $r DLI_SLAB_STORE_TILES=2
  run t26 $r DLI_GEMM_EXCLUDE=27,41,45
done
timeout -k 10 300 python3 scripts/bench_moe_tiles.py --batch 512 --which down > $O/moe_down_b512.log 2>&1
echo "rc[moe]=$?"
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o wave -- python3 bench.py --steps 1 --warmup 1 > $O/prof.log 2>&1
rc=$?; echo "rc[prof]=$rc"; [ $rc -eq 0 ] || exit $rc
python3 scripts/prof_summary.py $O/prof 30 --tail-ms 830 --gaps 5 > $O/wave_summary.txt 2>&1
rm -rf $O/prof
exit 0
