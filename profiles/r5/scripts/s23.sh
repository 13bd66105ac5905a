#!/bin/bash
# Session 23: a wave per row for prefill-sized norms (rows >= 1024); session 22: norm kernel with every row load issued up front (prefill add + RMSNorm was
# 1.6 TB/s), the fused decode attention's block-table window loaded without waiting on the
# context length. Kernel + engine tests, the driver's bench x2, a b512 wave summary.
set -u
O=gpurun_out/s23
mkdir -p $O
: > $O/bench.jsonl
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?;
         echo "rc[$name]=$rc"; tail -3 $O/$name.log; [ $rc -eq 0 ] || exit $rc; }
rec() { echo "{\"arm\": \"$1\", \"bench\": $(grep -h '^{"metric"' $O/$1.log)}" >> $O/bench.jsonl; }
step tests 600 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_kernels_gpu.py tests/test_engine_gpu.py -m gpu -k "norm or close_to_hf or graph_decode or mixed"
step bench1 300 python3 bench.py --gpus 1 --steps 20 --warmup 5
rec bench1
step bench2 300 python3 bench.py --gpus 1 --steps 20 --warmup 5
rec bench2
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o wave -- python3 bench.py --steps 1 --warmup 1 > $O/prof.log 2>&1
rc=$?; echo "rc[prof]=$rc"; [ $rc -eq 0 ] || exit $rc
python3 scripts/prof_summary.py $O/prof 30 --tail-ms 830 --gaps 5 > $O/wave_summary.txt 2>&1
rm -rf $O/prof
exit 0
