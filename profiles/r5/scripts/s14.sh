#!/bin/bash
# Session 14: the LM head's 16-column group maxima feeding the sampler (candidate path):
# GPU tests (bitwise logits, exact maxima, token identity), the driver bench with it on / off
# alternated x2, and a rocprofv3 wave summary with it on.
set -u
O=gpurun_out/s14
mkdir -p $O
: > $O/ab.jsonl
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?;
         echo "rc[$name]=$rc"; tail -3 $O/$name.log; [ $rc -eq 0 ] || exit $rc; }
run() { local arm=$1 r=$2; shift 2; timeout -k 10 300 env DLI_GEMM_AUTOTUNE_LOG=1 "$@" python3 bench.py --gpus 1 --steps 10 --warmup 3 > $O/${arm}_$r.log 2>&1;
        local rc=$?; echo "rc[$arm $r]=$rc"; [ $rc -eq 0 ] || { tail -20 $O/${arm}_$r.log; exit $rc; }
        echo "{\"arm\": \"$arm\", \"run\": $r, \"bench\": $(grep -h '^{"metric"' $O/${arm}_$r.log)}" >> $O/ab.jsonl
        grep -o '"value": [0-9.]*' $O/${arm}_$r.log; }
step tests 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_engine_gpu.py -k "group_max or sampl"
for r in 1 2; do
  run gmax $r DLI_AB=0
  run nogmax $r DLI_HEAD_GMAX=0
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o wave -- python3 bench.py --steps 1 --warmup 1 > $O/prof.log 2>&1
rc=$?; echo "rc[prof]=$rc"; [ $rc -eq 0 ] || exit $rc
python3 scripts/prof_summary.py $O/prof 30 --tail-ms 830 --gaps 5 > $O/wave_summary.txt 2>&1
rm -rf $O/prof
exit 0
