#!/bin/bash
# Session 34 (round 6): final HEAD validation after the prefill-attention fix — the whole GPU tier (serve-expert streamed apart),
# smoke(), the driver's bench command twice, batch 1 twice, and a rocprofv3 wave summary.
set -u
O=gpurun_out/r6s34
mkdir -p $O
: > $O/bench.jsonl
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?;
         echo "rc[$name]=$rc"; tail -3 $O/$name.log; [ $rc -eq 0 ] || exit $rc; }
rec() { echo "{\"arm\": \"$1\", \"bench\": $(grep -h '^{"metric"' $O/$1.log)}" >> $O/bench.jsonl; }
step tests 900 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests -m gpu --deselect tests/test_serving_gpu.py::test_serve_expert_on_gpu_through_master
echo "== serving"; timeout -k 10 600 python -u -m pytest -x -v -s --timeout 500 --timeout-method thread tests/test_serving_gpu.py::test_serve_expert_on_gpu_through_master > $O/serving.log 2>&1; rc=$?; echo "rc[serving]=$rc"; tail -2 $O/serving.log; [ $rc -eq 0 ] || exit $rc
step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"
step bench1 300 python3 bench.py --steps 20 --warmup 5
rec bench1
step b1_1 300 python3 bench.py --batch 1 --steps 8 --warmup 2
rec b1_1
step bench2 300 python3 bench.py --steps 20 --warmup 5
rec bench2
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o wave -- python3 bench.py --steps 1 --warmup 1 > $O/prof.log 2>&1
rc=$?; echo "rc[prof]=$rc"; [ $rc -eq 0 ] || exit $rc
python3 scripts/prof_summary.py $O/prof 30 --tail-ms 800 --gaps 5 > $O/wave_summary.txt 2>&1
rm -rf $O/prof
exit 0
