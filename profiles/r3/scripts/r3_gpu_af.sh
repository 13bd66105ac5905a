#!/bin/bash
# round 3, session AF: prefill autotune test + batch-512 wave profile at HEAD
set -o pipefail
mkdir -p gpurun_out/r3af
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r3af
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "rc[$name]=$rc"; tail -2 $O/$name.log | cut -c1-260; return $rc; }
run kern 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "prefill_autotune or gemv_skinny" &&
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null &&
run prof 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o b512 -- python bench.py --steps 2 --warmup 1 &&
python scripts/prof_summary.py $O/prof 40 --tail-ms 1600 > $O/prof_summary.txt && find $O/prof -name "*trace.csv" -delete
echo "end $(date +%T)"
