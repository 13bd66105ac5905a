#!/bin/bash
# round 3, session AM: wave-aggregated radix histograms in the sampler (tests + kernel times)
set -o pipefail
mkdir -p gpurun_out/r3am
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r3am
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "rc[$name]=$rc"; tail -2 $O/$name.log | cut -c1-300; return $rc; }
run kern 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "sampling or vocab_parallel or topk" &&
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null &&
run prof1 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof1 -o b1 -- python bench.py --steps 4 --warmup 1 --batch 1 &&
python scripts/prof_summary.py $O/prof1 25 --tail-ms 900 > $O/prof1_summary.txt && find $O/prof1 -name "*trace.csv" -delete &&
run prof512 500 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof512 -o b512 -- python bench.py --steps 2 --warmup 1 &&
python scripts/prof_summary.py $O/prof512 40 --tail-ms 1600 > $O/prof512_summary.txt && find $O/prof512 -name "*trace.csv" -delete &&
run b1 300 python -u bench.py --steps 16 --warmup 2 --batch 1 &&
run b512 400 python -u bench.py
echo "end $(date +%T)"
