#!/bin/bash
# Session 6 (re-entry after the container was re-created): the whole GPU tier on a fresh
# build, the driver's bench command, an attention-form A/B (one workgroup per item at b512),
# and a rocprofv3 wave summary at HEAD.
set -u
O=gpurun_out/s06
mkdir -p $O
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?;
         echo "rc[$name]=$rc"; tail -3 $O/$name.log; [ $rc -eq 0 ] || exit $rc; }
step tests 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu
step bench 300 python3 bench.py --gpus 1 --steps 20 --warmup 5
step wpi4 300 env DLI_DECODE_WPI=4 python3 bench.py --gpus 1 --steps 10 --warmup 3
step bench2 300 python3 bench.py --gpus 1 --steps 10 --warmup 3
for f in bench wpi4 bench2; do
  echo "{\"arm\": \"$f\", \"bench\": $(grep -h '^{"metric"' $O/$f.log)}" >> $O/bench.jsonl
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o wave -- python3 bench.py --steps 1 --warmup 1 > $O/prof.log 2>&1
rc=$?; echo "rc[prof]=$rc"; [ $rc -eq 0 ] || exit $rc
python3 scripts/prof_summary.py $O/prof 30 --tail-ms 830 --gaps 5 > $O/wave_summary.txt 2>&1
rm -rf $O/prof
exit 0
