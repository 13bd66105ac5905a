#!/bin/bash
# Session 11: where the skinny full-K tiles 60-62 land in the M = 512 decode landscape
# (every candidate plan printed), O / down / QKV.
set -u
O=gpurun_out/s11
mkdir -p $O
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?;
         echo "rc[$name]=$rc"; tail -3 $O/$name.log; [ $rc -eq 0 ] || exit $rc; }
step tiles 600 python3 scripts/bench_decode_tiles.py --m 512 --shapes o,down,qkv
exit 0
