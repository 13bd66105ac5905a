#!/bin/bash
# Session 7: the overlapped decode attention block (two half batches on two streams):
# its GPU tests, a probe of whether a replayed hipGraph runs independent branches
# concurrently, and a same-box A/B of the driver's bench (overlap off / on, alternated x2,
# autotune picks logged), plus sc1 (write-through) split-K slab stores for the 8-phase
# family (the decode down projection).
set -u
O=gpurun_out/s07
mkdir -p $O
: > $O/ab.jsonl
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?;
         echo "rc[$name]=$rc"; tail -3 $O/$name.log; [ $rc -eq 0 ] || exit $rc; }
run() { local arm=$1 r=$2; shift 2; timeout -k 10 300 env DLI_GEMM_AUTOTUNE_LOG=1 "$@" python3 bench.py --gpus 1 --steps 10 --warmup 3 > $O/${arm}_$r.log 2>&1;
        local rc=$?; echo "rc[$arm $r]=$rc"; [ $rc -eq 0 ] || { tail -20 $O/${arm}_$r.log; exit $rc; }
        echo "{\"arm\": \"$arm\", \"run\": $r, \"bench\": $(grep -h '^{"metric"' $O/${arm}_$r.log)}" >> $O/ab.jsonl
        grep -o '"value": [0-9.]*' $O/${arm}_$r.log; }
step probe 120 python3 scripts/probe_graph_concurrency.py
step tests 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_overlap_gpu.py
for r in 1 2; do
  run base $r DLI_AB=0
  run overlap $r DLI_DECODE_OVERLAP=1
done
run sc1_8p 1 DLI_SLAB_STORE_8P=2
run head45 1 DLI_GEMM_HEAD_4W=1
exit 0
