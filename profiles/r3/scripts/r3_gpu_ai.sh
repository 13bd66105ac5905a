#!/bin/bash
# round 3, session AI: other model families at HEAD (prefill autotune on): Llama-3-70B and
# Mixtral 8x7B at batch 512, plus the 70B with the prefill autotune off (A/B)
set -o pipefail
mkdir -p gpurun_out/r3ai
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r3ai
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "rc[$name]=$rc"; tail -2 $O/$name.log | cut -c1-300; return $rc; }
DLI_GEMM_AUTOTUNE_LOG=1 run mixtral 600 python -u bench.py --model mixtral-8x7b --steps 2 --warmup 1 &&
DLI_GEMM_AUTOTUNE_LOG=1 run l70 900 python -u bench.py --model llama3-70b --steps 2 --warmup 1 &&
DLI_TUNE_PREFILL=0 run l70_own 900 python -u bench.py --model llama3-70b --steps 2 --warmup 1
echo "end $(date +%T)"
