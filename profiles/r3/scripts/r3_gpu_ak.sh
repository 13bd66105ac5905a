#!/bin/bash
# round 3, session AK: full GPU validation at HEAD (pytest -m gpu, smoke, bench defaults)
set -o pipefail
mkdir -p gpurun_out/r3ak
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r3ak
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "rc[$name]=$rc"; tail -2 $O/$name.log | cut -c1-300; return $rc; }
run gpu_tests 900 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/ &&
run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" &&
run bench 400 python -u bench.py &&
run bench_b1 300 python -u bench.py --batch 1 --steps 16 --warmup 2
echo "end $(date +%T)"
