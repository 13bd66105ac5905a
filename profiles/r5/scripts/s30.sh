#!/bin/bash
# Session 30: where the time goes at 4 concurrent requests (M = 4 GEMV chain): wave summary.
set -u
O=gpurun_out/s30
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof4 -o wave -- python3 bench.py --batch 4 --steps 1 --warmup 1 > $O/prof4.log 2>&1
rc=$?; echo "rc[prof4]=$rc"; [ $rc -eq 0 ] || exit $rc
python3 scripts/prof_summary.py $O/prof4 16 --tail-ms 260 > $O/wave_summary_b4.txt 2>&1
rm -rf $O/prof4
cat $O/wave_summary_b4.txt
