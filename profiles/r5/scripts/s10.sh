#!/bin/bash
# Session 10: skinny full-K tiles 60-62 (gemm_sk.hip): GPU tests, the M = 512 decode
# landscape of the O / down / QKV / gate-up projections, and the driver bench with the new
# tiles in the decode autotune vs excluded (alternated x2, autotune picks logged).
set -u
O=gpurun_out/s10
mkdir -p $O
: > $O/ab.jsonl
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?;
         echo "rc[$name]=$rc"; tail -3 $O/$name.log; [ $rc -eq 0 ] || exit $rc; }
run() { local arm=$1 r=$2; shift 2; timeout -k 10 300 env DLI_GEMM_AUTOTUNE_LOG=1 "$@" python3 bench.py --gpus 1 --steps 10 --warmup 3 > $O/${arm}_$r.log 2>&1;
        local rc=$?; echo "rc[$arm $r]=$rc"; [ $rc -eq 0 ] || { tail -20 $O/${arm}_$r.log; exit $rc; }
        echo "{\"arm\": \"$arm\", \"run\": $r, \"bench\": $(grep -h '^{"metric"' $O/${arm}_$r.log)}" >> $O/ab.jsonl
        grep -o '"value": [0-9.]*' $O/${arm}_$r.log; }
step tests 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "skinny"
step tiles 600 python3 scripts/bench_decode_tiles.py --m 512 --shapes o,down,qkv,gate_up --top 10
for r in 1 2; do
  run sk $r DLI_AB=0
  run nosk $r DLI_GEMM_EXCLUDE=26,27,41,45,55,60,61,62
done
exit 0
