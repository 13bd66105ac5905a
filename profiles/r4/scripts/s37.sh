#!/bin/bash
# round 4, session 37: batch-1 gate/up on the 16-row SiLU GEMV grid (tile 29) — tests,
# isolated M = 1 sweep, b1 bench A/B alternated (29 excluded vs default)
set -o pipefail
R=$(pwd); O=$R/gpurun_out/r4s37; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "rc[$name]=$rc"; grep -h '"value"' $O/$name.log | cut -c90-330; tail -1 $O/$name.log | cut -c1-200; return $rc; }
step() { run "$@"; local rc=$?; [ $rc -le 1 ] || { echo "stop after rc=$rc"; exit $rc; }; }
step gemv_tests 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "gemv_skinny"
step sweep 300 python -u scripts/gemv_sweep.py --m 1 --out $O/gemv_sweep_m1.jsonl
grep gate_up $O/gemv_sweep_m1.jsonl | sort -t: -k9 | cut -c1-200
for r in 1 2; do
  step b1_no29_$r 300 env DLI_GEMM_EXCLUDE=26,27,29,41,45 DLI_GEMM_AUTOTUNE_LOG=1 python -u bench.py --batch 1 --steps 3 --warmup 1
  step b1_def_$r 300 env DLI_GEMM_AUTOTUNE_LOG=1 python -u bench.py --batch 1 --steps 3 --warmup 1
done
grep -h "28672" $O/b1_def_1.log | head -5
echo "end $(date +%T)"
