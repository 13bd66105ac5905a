#!/bin/bash
# round 4, session 24: full GPU test tier + smoke + bench (b512, b1) at HEAD
set -o pipefail
R=$(pwd); O=$R/gpurun_out/r4s24; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "rc[$name]=$rc"; tail -2 $O/$name.log | cut -c1-300; return $rc; }
step() { run "$@"; local rc=$?; [ $rc -le 1 ] || { echo "stop after rc=$rc"; exit $rc; }; }
step gpu_tests 900 python -u -m pytest -m gpu -v --timeout 300 --timeout-method thread tests/
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step bench 400 python -u bench.py --steps 5 --warmup 2
step bench_b1 400 python -u bench.py --batch 1 --steps 3 --warmup 1
echo "end $(date +%T)"
