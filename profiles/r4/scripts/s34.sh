#!/bin/bash
# round 4, session 34: two-phase sampler at batch 512 (DLI_SAMPLE_SPLIT_MAX_B=512) — tests,
# kernel times in the wave, bench A/B alternated
set -o pipefail
R=$(pwd); O=$R/gpurun_out/r4s34; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "rc[$name]=$rc"; grep -h '"value"' $O/$name.log | cut -c90-200; tail -1 $O/$name.log | cut -c1-200; return $rc; }
step() { run "$@"; local rc=$?; [ $rc -le 1 ] || { echo "stop after rc=$rc"; exit $rc; }; }
step smp_tests 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "sampl"
cd /tmp && export TMPDIR=/tmp
step prof512 600 env DLI_SAMPLE_SPLIT_MAX_B=512 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p -o run -- python3 $R/bench.py --steps 1 --warmup 1
cd $R
python3 scripts/prof_summary.py $O/p 40 --tail-ms 800 > $O/wave512.txt; rm -rf $O/p
grep -i "sampl" $O/wave512.txt
for r in 1 2; do
  step base_$r 400 python -u bench.py --steps 5 --warmup 2
  step split512_$r 400 env DLI_SAMPLE_SPLIT_MAX_B=512 python -u bench.py --steps 5 --warmup 2
done
echo "end $(date +%T)"
