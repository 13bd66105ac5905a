#!/bin/bash
# round 4, session 27: HEAD validation — GPU tests, smoke, bench, the b512 wave's kernel
# summary (rocprofv3, csv), and config 2 end to end through the public API (4,096 requests
# at concurrency 1,024, then 16 at concurrency 1)
set -o pipefail
R=$(pwd); O=$R/gpurun_out/r4s27; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "rc[$name]=$rc"; tail -2 $O/$name.log | cut -c1-300; return $rc; }
step() { run "$@"; local rc=$?; [ $rc -le 1 ] || { echo "stop after rc=$rc"; exit $rc; }; }
step gpu_tests 900 python -u -m pytest -m gpu -v --timeout 300 --timeout-method thread tests/
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step bench 400 python -u bench.py --steps 5 --warmup 2
cd /tmp && export TMPDIR=/tmp
step prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/llama_b512 -o run -- python3 $R/bench.py --steps 1 --warmup 1
cd $R
python3 scripts/prof_summary.py $O/llama_b512 60 > $O/llama_b512.all.txt
python3 scripts/prof_summary.py $O/llama_b512 60 --tail-ms 800 --gaps 10 > $O/llama_b512.wave.txt
find $O/llama_b512 -name "*kernel_stats.csv" -exec cp {} $O/llama_b512.stats.csv \;
rm -rf $O/llama_b512
step e2e 900 bash scripts/serve_e2e.sh 4096 1024 512 aiohttp
cp gpurun_out/e2e_*.json $O/ 2>/dev/null
echo "end $(date +%T)"
