#!/bin/bash
# Session 8: prefill-sized projection GEMMs per shape and plan (is the O projection the slow
# one?), and the fixed graph-concurrency probe.
set -u
O=gpurun_out/s08
mkdir -p $O
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?;
         echo "rc[$name]=$rc"; tail -3 $O/$name.log; [ $rc -eq 0 ] || exit $rc; }
step probe 120 python3 scripts/probe_graph_concurrency.py
step prefill 400 python3 scripts/bench_prefill_gemm.py --tiles 22,34,41,45 --splits 1,2
exit 0
