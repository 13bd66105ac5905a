#!/bin/bash
# Session 24 (round 6): the Mixtral gate/up GEMM reading its token rows through the permutation
# (dli_gemm_grouped_gather: no moe_gather copy) — GPU tests, the Mixtral b512 wave trace, and Mixtral b512
# runs (4 timed waves each) for the record.
set -u
O=gpurun_out/r6s24
mkdir -p $O
: > $O/bench.jsonl
PT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 700 $PT tests/test_kernels_gpu.py tests/test_engine_gpu.py tests/test_parallel_gpu.py -k "moe or router or gate or mixtral or expert or add_rmsnorm or combine or permutation or grouped" > $O/tests.log 2>&1
rc=$?; echo "rc[tests]=$rc"; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o wave -- python3 bench.py --model mixtral-8x7b --steps 1 --warmup 1 > $O/prof.log 2>&1
rc=$?; echo "rc[prof]=$rc"; [ $rc -eq 0 ] || exit $rc
python3 scripts/prof_summary.py $O/prof 30 --tail-ms 2000 --gaps 5 > $O/wave_summary.txt 2>&1
head -22 $O/wave_summary.txt
rm -rf $O/prof
for i in 1 2; do
  timeout -k 10 500 python3 bench.py --model mixtral-8x7b --steps 4 --warmup 1 > $O/mixtral_$i.log 2>&1
  rc=$?; echo "rc[mixtral_$i]=$rc"; [ $rc -eq 0 ] || exit $rc
  echo "{\"arm\": \"mixtral_$i\", \"bench\": $(grep -h '^{"metric"' $O/mixtral_$i.log)}" >> $O/bench.jsonl
  tail -1 $O/mixtral_$i.log
done
exit 0
