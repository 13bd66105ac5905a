#!/bin/bash
# Session 38: smoke() and the GEMV / engine decode tests on the final library build.
set -u
O=gpurun_out/s38
mkdir -p $O
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; echo "rc[smoke]=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py -x -q -m gpu -k "gemv or prologue or residual or deferred or graph_decode" > $O/tests.log 2>&1; rc=$?; echo "rc[tests]=$rc"; tail -1 $O/tests.log
exit $rc
