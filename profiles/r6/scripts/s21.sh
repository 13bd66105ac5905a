#!/bin/bash
# Session 21 (round 6): small decode kernels with every load issued before any use — the
# RMSNorm (+ residual add) kernel, the MoE combine of fp16 slabs (both top-2 picks at once)
# and the MoE row gather — kernel / engine / parallel GPU tests, the Mixtral b512 trace, and
# the Llama driver bench as a check.
set -u
O=gpurun_out/r6s21
mkdir -p $O
PT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 700 $PT tests/test_kernels_gpu.py tests/test_engine_gpu.py tests/test_parallel_gpu.py > $O/tests.log 2>&1
rc=$?; echo "rc[tests]=$rc"; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o wave -- python3 bench.py --model mixtral-8x7b --steps 1 --warmup 1 > $O/prof.log 2>&1
rc=$?; echo "rc[prof]=$rc"; [ $rc -eq 0 ] || exit $rc
python3 scripts/prof_summary.py $O/prof 30 --tail-ms 2000 --gaps 5 > $O/wave_summary.txt 2>&1
head -20 $O/wave_summary.txt
rm -rf $O/prof
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1
rc=$?; echo "rc[bench]=$rc"; tail -1 $O/bench.log
exit $rc
