#!/bin/bash
# round 4, session 18: two-barrier 4-wave GEMM — barrier placements 19/103 (45), 25/111 (49),
# 25/end (50), + deep W ring (51), tile order GM 8 (52) / none (53); then the headline bench
# A/B: prefill autotune with / without the 4-wave tile, tile 45 in the decode autotune
set -o pipefail
R=$(pwd); O=$R/gpurun_out/r4s18; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "rc[$name]=$rc"; grep -h '"value"' $O/$name.log | cut -c1-200; tail -1 $O/$name.log | cut -c1-200; return $rc; }
step() { run "$@"; local rc=$?; [ $rc -le 1 ] || { echo "stop after rc=$rc"; exit $rc; }; }
step t4w 300 env DLI_TEST_4W_TILES=45,49,50,51,52,53 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "4wave"
step gemm_sq 400 python -u scripts/bench_gemm8p.py --only sq --tiles 22,41,45,49,50,51,52,53 --out $O/gemm_sq.json
step gemm_prefill 500 python -u scripts/bench_gemm8p.py --only prefill --tiles 22,45,49,50,51,52 --out $O/gemm_prefill.json
step bench_default 400 python -u bench.py
step bench_no4w 400 env DLI_GEMM_PREFILL_4W=0 python -u bench.py
step bench_45decode 400 env DLI_GEMM_EXCLUDE=26,27,41,49,50,51,52,53 DLI_GEMM_AUTOTUNE_LOG=1 python -u bench.py
step bench_default2 400 python -u bench.py
echo "end $(date +%T)"
