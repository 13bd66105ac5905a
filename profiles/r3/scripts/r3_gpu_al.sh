#!/bin/bash
# round 3, session AL: batch-1 rocprof summary at HEAD
set -o pipefail
mkdir -p gpurun_out/r3al
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r3al
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "rc[$name]=$rc"; tail -2 $O/$name.log | cut -c1-300; return $rc; }
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null &&
run prof 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o b1 -- python bench.py --steps 4 --warmup 1 --batch 1 &&
python scripts/prof_summary.py $O/prof 25 --tail-ms 900 > $O/prof_summary.txt && find $O/prof -name "*trace.csv" -delete &&
run b1 300 python -u bench.py --steps 16 --warmup 2 --batch 1
echo "end $(date +%T)"
