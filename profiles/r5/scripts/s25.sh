#!/bin/bash
# Session 25: stream-K (tile 60) without cache-wide fences (sc1 hand-over): kernel tests, then
# isolated cold-weight timings of every candidate for the M = 512 gate/up and LM head.
set -u
O=gpurun_out/s25
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_kernels_gpu.py -m gpu -k "stream_k" > $O/tests.log 2>&1; rc=$?; echo "rc_tests=$rc"; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 scripts/bench_decode_tiles.py --m 512 --shapes gate_up,head --top 4 > $O/tiles.jsonl 2> $O/tiles.err; echo "rc=$?"
cat $O/tiles.jsonl
