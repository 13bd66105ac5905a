#!/bin/bash
# Session 13: the 4-wave tile 34 out of the decode autotune (new default) vs in it (round-4
# list), alternated x3 on one box with the driver's command, autotune picks logged.
set -u
O=gpurun_out/s13
mkdir -p $O
: > $O/ab.jsonl
run() { local arm=$1 r=$2; shift 2; timeout -k 10 300 env DLI_GEMM_AUTOTUNE_LOG=1 "$@" python3 bench.py --gpus 1 --steps 10 --warmup 3 > $O/${arm}_$r.log 2>&1;
        local rc=$?; echo "rc[$arm $r]=$rc"; [ $rc -eq 0 ] || { tail -20 $O/${arm}_$r.log; exit $rc; }
        echo "{\"arm\": \"$arm\", \"run\": $r, \"bench\": $(grep -h '^{"metric"' $O/${arm}_$r.log)}" >> $O/ab.jsonl
        grep -o '"value": [0-9.]*' $O/${arm}_$r.log; }
for r in 1 2 3; do
  run no34 $r DLI_AB=0
  run with34 $r DLI_GEMM_EXCLUDE=26,27,41,45,55
done
exit 0
