#!/bin/bash
# Session 11 (round 6): batch-1 decode with the O-projection weights streamed into the
# Infinity Cache beside the latency-bound attention kernel (side-stream fork / join in the
# decode graph) — engine GPU tests, then a same-box alternated A/B of bench.py --batch 1, and
# a rocprofv3 wave of the new default.
set -u
O=gpurun_out/r6s11
mkdir -p $O
: > $O/bench.jsonl
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?;
         echo "rc[$name]=$rc"; tail -2 $O/$name.log; [ $rc -eq 0 ] || exit $rc; }
rec() { echo "{\"arm\": \"$1\", \"bench\": $(grep -h '^{"metric"' $O/$1.log)}" >> $O/bench.jsonl; }
PT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
step engine 600 $PT tests/test_engine_gpu.py
step b1_pf_1 240 python3 -u bench.py --batch 1 --steps 8 --warmup 2
rec b1_pf_1
step b1_off_1 240 env DLI_B1_PREFETCH=0 python3 -u bench.py --batch 1 --steps 8 --warmup 2
rec b1_off_1
step b1_pf_2 240 python3 -u bench.py --batch 1 --steps 8 --warmup 2
rec b1_pf_2
step b1_off_2 240 env DLI_B1_PREFETCH=0 python3 -u bench.py --batch 1 --steps 8 --warmup 2
rec b1_off_2
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof1 -o wave -- python3 bench.py --batch 1 --steps 1 --warmup 1 > $O/prof1.log 2>&1
rc=$?; echo "rc[prof1]=$rc"; [ $rc -eq 0 ] || exit $rc
python3 scripts/prof_summary.py $O/prof1 25 --tail-ms 200 --gaps 5 > $O/wave_summary_b1.txt 2>&1
rm -rf $O/prof1
exit 0
