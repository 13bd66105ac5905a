#!/bin/bash
# Session 4: the whole GPU test tier on the refactored GEMM sources (per-family translation
# units, no library backend), the driver's bench command, and a rocprofv3 wave profile.
set -u
O=gpurun_out/s04
mkdir -p $O
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?;
         echo "rc[$name]=$rc"; tail -3 $O/$name.log; [ $rc -eq 0 ] || exit $rc; }
step tests 1500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu
step bench 300 python3 bench.py --gpus 1 --steps 20 --warmup 5
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step prof 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o wave -- python3 bench.py --steps 1 --warmup 1
exit 0
