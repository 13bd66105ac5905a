#!/bin/bash
# Session 18 (round 6): the fused MoE gate in the Mixtral b512 wave — a rocprofv3 kernel
# trace (moe_router_kernel against the GEMM + split-K reduce + route kernels it replaces,
# s16), then a longer alternated A/B (4 timed waves per run).
set -u
O=gpurun_out/r6s18
mkdir -p $O
: > $O/bench.jsonl
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?;
         echo "rc[$name]=$rc"; tail -1 $O/$name.log; [ $rc -eq 0 ] || exit $rc; }
rec() { echo "{\"arm\": \"$1\", \"bench\": $(grep -h '^{"metric"' $O/$1.log)}" >> $O/bench.jsonl; }
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o wave -- python3 bench.py --model mixtral-8x7b --steps 1 --warmup 1 > $O/prof.log 2>&1
rc=$?; echo "rc[prof]=$rc"; [ $rc -eq 0 ] || exit $rc
python3 scripts/prof_summary.py $O/prof 30 --tail-ms 2000 --gaps 5 > $O/wave_summary.txt 2>&1
head -24 $O/wave_summary.txt
rm -rf $O/prof








exit 0
