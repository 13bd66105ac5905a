#!/bin/bash
# Session 2: serving/launcher GPU tests, then the driver-form multi-rank bench (spawned ranks,
# same GPU) beside the single engine on the same box.
set -u
O=gpurun_out/s02
mkdir -p $O
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?;
         echo "rc[$name]=$rc"; tail -3 $O/$name.log; [ $rc -eq 0 ] || exit $rc; }
step tests 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_serving_gpu.py tests/test_parallel_gpu.py tests/test_ipc_gpu.py
step pp2_spawn 600 env DLI_SAME_DEVICE=1 python3 bench.py --gpus 2
step single 300 python3 bench.py
grep -h '^{"metric"' $O/pp2_spawn.log $O/single.log > $O/bench.jsonl
exit 0
