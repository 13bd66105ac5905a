#!/bin/bash
# round 3, session AH: two-phase small-batch sampler + LDS hand-off of the new k/v row in the
# small-batch fused decode attention (tests + batch-1 A/Bs + rocprof summary)
set -o pipefail
mkdir -p gpurun_out/r3ah
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r3ah
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "rc[$name]=$rc"; tail -2 $O/$name.log | cut -c1-300; return $rc; }
run kern 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "sampling or vocab_parallel or attention" &&
run kern_nolds 300 env DLI_ATTN_KV_LDS=0 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "fused_rope_attention" &&
run b1_new1 300 python -u bench.py --steps 16 --warmup 2 --batch 1 &&
DLI_SAMPLE_SPLIT=0 DLI_ATTN_KV_LDS=0 run b1_old1 300 python -u bench.py --steps 16 --warmup 2 --batch 1 &&
DLI_SAMPLE_SPLIT=0 run b1_nosmp1 300 python -u bench.py --steps 16 --warmup 2 --batch 1 &&
run b1_new2 300 python -u bench.py --steps 16 --warmup 2 --batch 1 &&
DLI_SAMPLE_SPLIT=0 DLI_ATTN_KV_LDS=0 run b1_old2 300 python -u bench.py --steps 16 --warmup 2 --batch 1 &&
DLI_ATTN_KV_LDS=0 run b1_nolds 300 python -u bench.py --steps 16 --warmup 2 --batch 1 &&
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null &&
run prof 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o b1 -- python bench.py --steps 4 --warmup 1 --batch 1 &&
python scripts/prof_summary.py $O/prof 25 --tail-ms 900 > $O/prof_summary.txt && find $O/prof -name "*trace.csv" -delete
echo "end $(date +%T)"
