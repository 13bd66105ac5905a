#!/bin/bash
# Session 35 (round 6): Mixtral 8x7B b512 on the final HEAD (prefill attention fix included)
# — the driver-form bench twice and a wave summary.
set -u
O=gpurun_out/r6s35
mkdir -p $O
: > $O/bench.jsonl
for i in 1 2; do
  timeout -k 10 500 python3 bench.py --model mixtral-8x7b --steps 4 --warmup 1 > $O/mixtral_$i.log 2>&1
  rc=$?; echo "rc[mixtral_$i]=$rc"; [ $rc -eq 0 ] || exit $rc
  echo "{\"arm\": \"mixtral_$i\", \"bench\": $(grep -h '^{"metric"' $O/mixtral_$i.log)}" >> $O/bench.jsonl
  tail -1 $O/mixtral_$i.log | cut -c1-200
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o wave -- python3 bench.py --model mixtral-8x7b --steps 1 --warmup 1 > $O/prof.log 2>&1
rc=$?; echo "rc[prof]=$rc"; [ $rc -eq 0 ] || exit $rc
python3 scripts/prof_summary.py $O/prof 30 --tail-ms 2000 --gaps 5 > $O/wave_summary.txt 2>&1
head -12 $O/wave_summary.txt | cut -c1-120
rm -rf $O/prof
exit 0
