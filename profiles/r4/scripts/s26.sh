#!/bin/bash
# round 4, session 26: s_memtime stamps in the two-barrier 4-wave GEMM (diagnostic tile 48)
set -o pipefail
R=$(pwd); O=$R/gpurun_out/r4s26; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python -u scripts/stamp_gemm4w.py --out $O/stamps.jsonl > $O/stamps.log 2>&1; rc=$?
echo "rc=$rc"; cat $O/stamps.log | tail -5 | cut -c1-900
