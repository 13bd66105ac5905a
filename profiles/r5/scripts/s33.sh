#!/bin/bash
# Session 33: same-box A/B of the prologue-width change at batch 1 and batch 4: ab_base/ =
# the previous commit (runtime branch over 2 / 4 row vectors), the tree = the template form.
set -u
O=gpurun_out/s33
mkdir -p $O
: > $O/ab.jsonl
R=$GRAFT_REPO_ROOT
run() { local name=$1 dir=$2; shift 2; echo "== $name"; (cd $dir && timeout -k 10 240 python3 bench.py "$@") > $O/$name.log 2>&1; local rc=$?;
        echo "rc[$name]=$rc"; [ $rc -eq 0 ] || exit $rc;
        echo "{\"arm\": \"$name\", \"bench\": $(grep -h '^{"metric"' $O/$name.log)}" >> $O/ab.jsonl; }
for i in 1 2; do
  run base_b1_$i $R/ab_base --batch 1 --steps 8 --warmup 2
  run new_b1_$i $R --batch 1 --steps 8 --warmup 2
done
run base_b4 $R/ab_base --batch 4 --steps 4 --warmup 1
run new_b4 $R --batch 4 --steps 4 --warmup 1
exit 0
