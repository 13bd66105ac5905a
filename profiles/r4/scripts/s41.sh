#!/bin/bash
# round 4, session 41: GPU tests and smoke after the M <= 2 heuristic moved to tile 29
set -o pipefail
R=$(pwd); O=$R/gpurun_out/r4s41; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "rc[$name]=$rc"; tail -1 $O/$name.log | cut -c1-200; return $rc; }
step() { run "$@"; local rc=$?; [ $rc -le 1 ] || { echo "stop after rc=$rc"; exit $rc; }; }
step gpu_tests 900 python -u -m pytest -m gpu -v --timeout 300 --timeout-method thread tests/
step smoke 300 python3 -u -c "import __graft_entry__ as g; g.smoke()"
step b1_noautotune 300 env DLI_GEMM_AUTOTUNE=0 python -u bench.py --batch 1 --steps 3 --warmup 1
echo "end $(date +%T)"
