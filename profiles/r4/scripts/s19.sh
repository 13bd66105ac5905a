#!/bin/bash
# round 4, session 19: headline bench A/B on one box — prefill autotune 8-phase vs the
# two-barrier 4-wave tile (45), and tile 45 also in the decode autotune
set -o pipefail
R=$(pwd); O=$R/gpurun_out/r4s19; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "rc[$name]=$rc"; grep -h '"value"' $O/$name.log | cut -c1-200; return $rc; }
step() { run "$@"; local rc=$?; [ $rc -le 1 ] || { echo "stop after rc=$rc"; exit $rc; }; }
step bench_default 400 python -u bench.py
step bench_no4w 400 env DLI_GEMM_PREFILL_4W=0 python -u bench.py
step bench_45decode 400 env DLI_GEMM_EXCLUDE=26,27,41,49,50,51 DLI_GEMM_AUTOTUNE_LOG=1 python -u bench.py
step bench_default2 400 python -u bench.py
echo "end $(date +%T)"
