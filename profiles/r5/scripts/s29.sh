#!/bin/bash
# Session 29: the driver's forms once more after the bench.py heartbeat: bench (1 GPU),
# batch 1, smoke(), and the spawned same-GPU pp2 (plain `python bench.py --gpus 2`).
set -u
O=gpurun_out/s29
mkdir -p $O
: > $O/bench.jsonl
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.log 2> $O/$name.err; local rc=$?;
         echo "rc[$name]=$rc"; tail -2 $O/$name.log; tail -2 $O/$name.err; [ $rc -eq 0 ] || exit $rc; }
rec() { echo "{\"arm\": \"$1\", \"bench\": $(grep -h '^{"metric"' $O/$1.log)}" >> $O/bench.jsonl; }
step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()"
step bench 300 python3 bench.py --gpus 1 --steps 20 --warmup 5
rec bench
step b1 300 python3 bench.py --batch 1 --steps 8 --warmup 2
rec b1
step pp2 600 env DLI_SAME_DEVICE=1 python3 bench.py --gpus 2 --steps 2 --warmup 1
rec pp2
exit 0
