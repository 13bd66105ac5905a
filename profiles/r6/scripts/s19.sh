#!/bin/bash
# Session 19 (round 6): the fused MoE gate as one workgroup per token (the wave-per-token
# form took 14.9 us in s18) — router / MoE / engine GPU tests, then the Mixtral b512 kernel
# trace.
set -u
O=gpurun_out/r6s19
mkdir -p $O
PT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 600 $PT tests/test_kernels_gpu.py tests/test_engine_gpu.py tests/test_parallel_gpu.py -k "moe or router or mixtral or expert" > $O/tests.log 2>&1
rc=$?; echo "rc[tests]=$rc"; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o wave -- python3 bench.py --model mixtral-8x7b --steps 1 --warmup 1 > $O/prof.log 2>&1
rc=$?; echo "rc[prof]=$rc"; [ $rc -eq 0 ] || exit $rc
python3 scripts/prof_summary.py $O/prof 30 --tail-ms 2000 --gaps 5 > $O/wave_summary.txt 2>&1
head -20 $O/wave_summary.txt
rm -rf $O/prof
exit 0
