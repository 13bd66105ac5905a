#!/bin/bash
# Session 9: the persistent 4-wave tile (55): its GPU tests, the prefill GEMM sweep against
# tiles 22 / 45, and the driver bench with 55 in the prefill autotune vs without (alternated).
set -u
O=gpurun_out/s09
mkdir -p $O
: > $O/ab.jsonl
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?;
         echo "rc[$name]=$rc"; tail -3 $O/$name.log; [ $rc -eq 0 ] || exit $rc; }
run() { local arm=$1 r=$2; shift 2; timeout -k 10 300 env DLI_GEMM_AUTOTUNE_LOG=1 "$@" python3 bench.py --gpus 1 --steps 10 --warmup 3 > $O/${arm}_$r.log 2>&1;
        local rc=$?; echo "rc[$arm $r]=$rc"; [ $rc -eq 0 ] || { tail -20 $O/${arm}_$r.log; exit $rc; }
        echo "{\"arm\": \"$arm\", \"run\": $r, \"bench\": $(grep -h '^{"metric"' $O/${arm}_$r.log)}" >> $O/ab.jsonl
        grep -o '"value": [0-9.]*' $O/${arm}_$r.log; }
step tests 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "persistent or gemm_4wave_256"
step prefill 400 python3 scripts/bench_prefill_gemm.py --tiles 22,45,55,45,55 --splits 1
for r in 1 2; do
  run persist $r DLI_AB=0
  run no55 $r DLI_GEMM_PREFILL_PERSIST=0
done
exit 0
