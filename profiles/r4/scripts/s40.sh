#!/bin/bash
# round 4, session 40: final HEAD check (tile 29, workspace retention) — all GPU tests, smoke,
# the driver's bench command twice, batch 1
set -o pipefail
R=$(pwd); O=$R/gpurun_out/r4s40; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "rc[$name]=$rc"; grep -h '"value"' $O/$name.log | cut -c90-260; tail -1 $O/$name.log | cut -c1-200; return $rc; }
step() { run "$@"; local rc=$?; [ $rc -le 1 ] || { echo "stop after rc=$rc"; exit $rc; }; }
step gpu_tests 900 python -u -m pytest -m gpu -v --timeout 300 --timeout-method thread tests/
step smoke 300 python3 -u -c "import __graft_entry__ as g; g.smoke()"
step driver_bench_1 600 python3 -u bench.py --gpus 1 --steps 20 --warmup 5
step driver_bench_2 600 python3 -u bench.py --gpus 1 --steps 20 --warmup 5
step b1 300 python -u bench.py --batch 1 --steps 3 --warmup 1
echo "end $(date +%T)"
