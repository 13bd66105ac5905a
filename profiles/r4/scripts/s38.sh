#!/bin/bash
# round 4, session 38: tile 29 (16-row SiLU GEMV) at M = 1..4 — full GPU tests, smoke, M = 2 / 4
# sweeps, b4 A/B (29 excluded vs default), b1 and the driver's bench command at HEAD
set -o pipefail
R=$(pwd); O=$R/gpurun_out/r4s38; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "rc[$name]=$rc"; grep -h '"value"' $O/$name.log | cut -c90-260; tail -1 $O/$name.log | cut -c1-200; return $rc; }
step() { run "$@"; local rc=$?; [ $rc -le 1 ] || { echo "stop after rc=$rc"; exit $rc; }; }
step gpu_tests 900 python -u -m pytest -m gpu -v --timeout 300 --timeout-method thread tests/
step smoke 300 python3 -u -c "import __graft_entry__ as g; g.smoke()"
step sweep_m2 300 python -u scripts/gemv_sweep.py --m 2 --out $O/gemv_sweep_m2.jsonl
step sweep_m4 300 python -u scripts/gemv_sweep.py --m 4 --out $O/gemv_sweep_m4.jsonl
grep gate_up $O/gemv_sweep_m2.jsonl $O/gemv_sweep_m4.jsonl | grep -E '"tile": (29|31|6),' | cut -c1-220
for r in 1 2; do
  step b4_no29_$r 300 env DLI_GEMM_EXCLUDE=26,27,29,41,45 DLI_GEMM_AUTOTUNE_LOG=1 python -u bench.py --batch 4 --steps 3 --warmup 1
  step b4_def_$r 300 env DLI_GEMM_AUTOTUNE_LOG=1 python -u bench.py --batch 4 --steps 3 --warmup 1
done
step b1_def 300 env DLI_GEMM_AUTOTUNE_LOG=1 python -u bench.py --batch 1 --steps 3 --warmup 1
step driver_bench 600 python3 -u bench.py --gpus 1 --steps 20 --warmup 5
grep -h "silu_mul" $O/b4_def_1.log $O/b4_no29_1.log | head -4
echo "end $(date +%T)"
