#!/bin/bash
# round 4, session 23: column-major MFMA order in the two-barrier 4-wave GEMM (46: weight
# operand reused for 8 consecutive MFMAs, the library's order) vs 45; then the decode
# autotune with / without tile 45, alternated three times (5 timed waves each)
set -o pipefail
R=$(pwd); O=$R/gpurun_out/r4s23; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "rc[$name]=$rc"; grep -h '"value"' $O/$name.log | cut -c100-200; tail -1 $O/$name.log | cut -c1-120; return $rc; }
step() { run "$@"; local rc=$?; [ $rc -le 1 ] || { echo "stop after rc=$rc"; exit $rc; }; }
step t4w 300 env DLI_TEST_4W_TILES=45,46 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "4wave"
step gemm_sq 400 python -u scripts/bench_gemm8p.py --only sq --tiles 22,45,46 --out $O/gemm_sq.json
step gemm_prefill 500 python -u scripts/bench_gemm8p.py --only prefill --tiles 22,45,46 --out $O/gemm_prefill.json
step gemm_decode 400 python -u scripts/bench_gemm8p.py --only b512 --tiles 22,34,45,46 --out $O/gemm_decode.json
for r in 1 2 3; do
  step base_$r 400 python -u bench.py --steps 5 --warmup 2
  step t45_$r 400 env DLI_GEMM_EXCLUDE=26,27,41 python -u bench.py --steps 5 --warmup 2
done
echo "end $(date +%T)"
