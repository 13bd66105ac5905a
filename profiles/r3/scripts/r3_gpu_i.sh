# round 3, GPU session I: default (batch-512 headline) bench with the graph-timed autotune,
# then batch 1 again.
set -o pipefail
mkdir -p gpurun_out/r3i
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r3i
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 $t "$@" 2>&1 | tee $O/$name.log; local rc=$?; echo "rc[$name]=$rc"; return $rc; }
DLI_GEMM_AUTOTUNE_LOG=1 run bdef 600 python -u bench.py --steps 3 --warmup 1 &&
DLI_GEMM_AUTOTUNE_LOG=1 run b1 300 python -u bench.py --steps 8 --warmup 1 --batch 1
echo "end $(date +%T)"
