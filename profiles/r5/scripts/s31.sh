#!/bin/bash
# Session 31: every candidate plan at M = 4 and M = 1 (cold weights) for the decode shapes.
set -u
O=gpurun_out/s31
mkdir -p $O
for m in 4 1; do
  timeout -k 10 300 python3 scripts/bench_decode_tiles.py --m $m --shapes gate_up,o,down,head --top 5 > $O/tiles_m$m.jsonl 2> $O/tiles_m$m.err; echo "rc_m$m=$?"
done
cat $O/tiles_m4.jsonl $O/tiles_m1.jsonl
