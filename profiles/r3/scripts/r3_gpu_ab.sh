# round 3, session AB: batch-1 latency at HEAD (bench + rocprof summary)
set -o pipefail
mkdir -p gpurun_out/r3ab
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r3ab
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "rc[$name]=$rc"; tail -1 $O/$name.log | cut -c1-260; return $rc; }
run b1a 300 python -u bench.py --steps 16 --warmup 2 --batch 1 &&
DLI_REDUCE_THREADS=256 run b1_r256 300 python -u bench.py --steps 16 --warmup 2 --batch 1 &&
run b1b 300 python -u bench.py --steps 16 --warmup 2 --batch 1 &&
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null &&
run prof 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o b1 -- python bench.py --steps 4 --warmup 1 --batch 1 &&
python scripts/prof_summary.py $O/prof 25 --tail-ms 900 > $O/prof_summary.txt && find $O/prof -name "*trace.csv" -delete
echo "end $(date +%T)"
