#!/bin/bash
# Session 3: GPU tests (fused batch-1 GEMV combine, serving, parallel), batch-1 A/B of the
# in-launch combine, the spawned pp2 bench and the single-engine bench on one box.
set -u
O=gpurun_out/s03
mkdir -p $O
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?;
         echo "rc[$name]=$rc"; tail -3 $O/$name.log; [ $rc -eq 0 ] || exit $rc; }
step tests 1100 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k "in_launch or gemv or add_rmsnorm" tests/test_serving_gpu.py tests/test_parallel_gpu.py tests/test_ipc_gpu.py tests/test_engine_gpu.py
step b1_fused 300 python3 bench.py --batch 1 --steps 8 --warmup 2
step b1_unfused 300 env DLI_GEMV_FUSED_NORM=0 python3 bench.py --batch 1 --steps 8 --warmup 2
step b1_fused2 300 python3 bench.py --batch 1 --steps 8 --warmup 2
step pp2_spawn 600 env DLI_SAME_DEVICE=1 python3 bench.py --gpus 2
step single 300 python3 bench.py
for f in b1_fused b1_unfused b1_fused2 pp2_spawn single; do
  echo "{\"arm\": \"$f\", \"bench\": $(grep -h '^{"metric"' $O/$f.log)}" >> $O/bench.jsonl
done
exit 0
