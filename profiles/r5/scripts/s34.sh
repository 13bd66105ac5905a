#!/bin/bash
# Session 34: one-row prologue GEMVs back on the runtime branch, several rows on the template
# form: GEMV tests, then batch 1 / batch 4 against ab_base/ (the commit before the change).
set -u
O=gpurun_out/s34
mkdir -p $O
: > $O/ab.jsonl
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_kernels_gpu.py tests/test_engine_gpu.py -m gpu -k "gemv or prologue or residual or deferred or batch_invariant" > $O/tests.log 2>&1; rc=$?; echo "rc[tests]=$rc"; tail -1 $O/tests.log; [ $rc -eq 0 ] || exit $rc
run() { local name=$1 dir=$2; shift 2; echo "== $name"; (cd $dir && timeout -k 10 240 python3 bench.py "$@") > $O/$name.log 2>&1; local rc=$?;
        echo "rc[$name]=$rc"; [ $rc -eq 0 ] || exit $rc;
        echo "{\"arm\": \"$name\", \"bench\": $(grep -h '^{"metric"' $O/$name.log)}" >> $O/ab.jsonl; }
run new_b1_1 $R --batch 1 --steps 8 --warmup 2
run base_b1_1 $R/ab_base --batch 1 --steps 8 --warmup 2
run new_b1_2 $R --batch 1 --steps 8 --warmup 2
run new_b4 $R --batch 4 --steps 4 --warmup 1
exit 0
