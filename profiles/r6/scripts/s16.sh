#!/bin/bash
# Session 16 (round 6): rocprofv3 kernel trace of a Mixtral 8x7B b512 wave (where the decode
# step's time goes besides the expert GEMMs).
set -u
O=gpurun_out/r6s16
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o wave -- python3 bench.py --model mixtral-8x7b --steps 1 --warmup 1 > $O/prof.log 2>&1
rc=$?; echo "rc[prof]=$rc"; tail -2 $O/prof.log; [ $rc -eq 0 ] || exit $rc
python3 scripts/prof_summary.py $O/prof 30 --tail-ms 2000 --gaps 5 > $O/wave_summary.txt 2>&1
head -40 $O/wave_summary.txt
rm -rf $O/prof
exit 0
