# round 3, GPU session D: batch-1 path. Every decode-plan candidate at M = 1 (MFMA tiles and
# the weight-streaming GEMV), then a rocprof kernel summary of a batch-1 bench.
set -o pipefail
mkdir -p gpurun_out/r3d
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r3d
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "rc[$name]=$rc"; tail -3 $O/$name.log; return $rc; }
run tiles_m1 600 python scripts/bench_decode_tiles.py --m 1 --shapes qkv,o,gate_up,down --top 6 &&
DLI_GEMM_AUTOTUNE_LOG=1 run b1_tune 600 python bench.py --steps 8 --warmup 1 --batch 1 &&
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null &&
run prof_b1 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_b1 -o b1 -- python bench.py --steps 2 --warmup 1 --batch 1 &&
python scripts/prof_summary.py $O/prof_b1 30 --tail-ms 500 --gaps 12 > $O/prof_b1_summary.txt; find $O/prof_b1 -name "*trace.csv" -delete
echo "end $(date +%T)"
