#!/bin/bash
# Session 35: HEAD validation after the tiny-batch prologue fix: the GPU tier
# (serve-expert streamed separately), smoke(), the driver's bench x2, batch 1 x2, and rocprofv3
# wave summaries of both.
set -u
O=gpurun_out/s35
mkdir -p $O
: > $O/bench.jsonl
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?;
         echo "rc[$name]=$rc"; tail -3 $O/$name.log; [ $rc -eq 0 ] || exit $rc; }
rec() { echo "{\"arm\": \"$1\", \"bench\": $(grep -h '^{"metric"' $O/$1.log)}" >> $O/bench.jsonl; }
step tests 900 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests -m gpu --deselect tests/test_serving_gpu.py::test_serve_expert_on_gpu_through_master
echo "== serving"; timeout -k 10 600 python -u -m pytest -x -v -s --timeout 500 --timeout-method thread tests/test_serving_gpu.py::test_serve_expert_on_gpu_through_master > $O/serving.log 2>&1; rc=$?; echo "rc[serving]=$rc"; tail -2 $O/serving.log; [ $rc -eq 0 ] || exit $rc
step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"
step bench1 300 python3 bench.py --gpus 1 --steps 20 --warmup 5
rec bench1
step b1_1 300 python3 bench.py --batch 1 --steps 8 --warmup 2
rec b1_1
step b4 240 python3 bench.py --batch 4 --steps 4 --warmup 1
rec b4
exit 0
