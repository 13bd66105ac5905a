#!/bin/bash
# round 4, session 32: GQA head packing in the short-prompt prefill attention kernel — GPU
# tests (bit-identical to unpacked, vs fp32 reference; paged chunks), full kernel tier, kernel
# summary of the prefill attention, bench A/B (packing on / off)
set -o pipefail
R=$(pwd); O=$R/gpurun_out/r4s32; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "rc[$name]=$rc"; grep -h '"value"' $O/$name.log | cut -c90-200; tail -1 $O/$name.log | cut -c1-200; return $rc; }
step() { run "$@"; local rc=$?; [ $rc -le 1 ] || { echo "stop after rc=$rc"; exit $rc; }; }
step attn_tests 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "prefill_attention"
step kernels 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py tests/test_engine_gpu.py
step bench_pack 400 python -u bench.py --steps 5 --warmup 2
step bench_nopack 400 env DLI_PREFILL_PACK=0 python -u bench.py --steps 5 --warmup 2
step bench_pack2 400 python -u bench.py --steps 5 --warmup 2
cd /tmp && export TMPDIR=/tmp
step prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p -o run -- python3 $R/bench.py --steps 1 --warmup 1
cd $R
python3 scripts/prof_summary.py $O/p 40 --tail-ms 800 > $O/wave.txt; rm -rf $O/p
grep prefill_attn $O/wave.txt
echo "end $(date +%T)"
