# round 3, session S: Llama-3-70B batch-512 decode profile (per-kernel times of the 8192-wide
# shapes) with the autotune log
set -o pipefail
mkdir -p gpurun_out/r3s
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r3s
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "rc[$name]=$rc"; tail -1 $O/$name.log | cut -c1-300; return $rc; }
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null &&
DLI_GEMM_AUTOTUNE_LOG=1 run prof70 1000 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof70 -o b512 -- python -u bench.py --model llama3-70b --steps 1 --warmup 1 &&
python scripts/prof_summary.py $O/prof70 30 --tail-ms 5000 > $O/prof70_summary.txt && find $O/prof70 -name "*trace.csv" -delete
echo "end $(date +%T)"
