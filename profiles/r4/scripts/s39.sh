#!/bin/bash
# round 4, session 39: after keeping replaced GEMM workspaces alive (a decode graph captured
# before the prefill autotune grew the workspace wrote into a freed buffer: batch-4 bench
# aborted in session 38) — engine GPU tests, b4 A/B (tile 29 excluded vs default), b1, the
# driver's bench command
set -o pipefail
R=$(pwd); O=$R/gpurun_out/r4s39; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "rc[$name]=$rc"; grep -h '"value"' $O/$name.log | cut -c90-260; tail -1 $O/$name.log | cut -c1-200; return $rc; }
step() { run "$@"; local rc=$?; [ $rc -le 1 ] || { echo "stop after rc=$rc"; exit $rc; }; }
step engine_tests 600 python -u -m pytest -m gpu -v --timeout 300 --timeout-method thread tests/test_engine_gpu.py
for r in 1 2; do
  step b4_no29_$r 300 env DLI_GEMM_EXCLUDE=26,27,29,41,45 DLI_GEMM_AUTOTUNE_LOG=1 python -u bench.py --batch 4 --steps 3 --warmup 1
  step b4_def_$r 300 env DLI_GEMM_AUTOTUNE_LOG=1 python -u bench.py --batch 4 --steps 3 --warmup 1
done
step b1_def_1 300 env DLI_GEMM_AUTOTUNE_LOG=1 python -u bench.py --batch 1 --steps 3 --warmup 1
step b1_def_2 300 python -u bench.py --batch 1 --steps 3 --warmup 1
step driver_bench 600 python3 -u bench.py --gpus 1 --steps 20 --warmup 5
grep -h "silu_mul" $O/b4_def_1.log | head -3
echo "end $(date +%T)"
