# round 3, GPU session L: fused decode attention A/B (prologue order: HEAD a5cbcc0 vs tree),
# and split-2 slabs vs bf16 rows (splits 0) at B = 512.
set -o pipefail
mkdir -p gpurun_out/r3l
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r3l
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "rc[$name]=$rc"; cat $O/$name.log | grep '^{' | cut -c1-200; return $rc; }
run ab_order 300 python -u scripts/bench_fused_attn.py --lib ab/libattention_decode_a5cbcc0.so --B 512,64 &&
run spl0 300 python -u scripts/bench_fused_attn.py --splits 0 --B 512,64 &&
run spl4 300 python -u scripts/bench_fused_attn.py --splits 4 --B 512
echo "end $(date +%T)"
