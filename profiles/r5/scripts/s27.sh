#!/bin/bash
# Session 27: batch-1 attention + O projection in one launch (dli_decode_attention_o): kernel
# and engine tests, batch-1 bench with it on / off alternated, a batch-1 wave summary.
set -u
O=gpurun_out/s27
mkdir -p $O
: > $O/bench.jsonl
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?;
         echo "rc[$name]=$rc"; tail -3 $O/$name.log; [ $rc -eq 0 ] || exit $rc; }
rec() { echo "{\"arm\": \"$1\", \"bench\": $(grep -h '^{"metric"' $O/$1.log)}" >> $O/bench.jsonl; }
step tests 600 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_kernels_gpu.py tests/test_engine_gpu.py -m gpu -k "attention_o or fused_rope or gemv or deferred or batch_invariant or graph_decode or loopback"
step on_1 300 python3 bench.py --batch 1 --steps 8 --warmup 2
rec on_1
step off_1 300 env DLI_ATTN_O=0 python3 bench.py --batch 1 --steps 8 --warmup 2
rec off_1
step on_2 300 python3 bench.py --batch 1 --steps 8 --warmup 2
rec on_2
step off_2 300 env DLI_ATTN_O=0 python3 bench.py --batch 1 --steps 8 --warmup 2
rec off_2
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof1 -o wave -- python3 bench.py --batch 1 --steps 1 --warmup 1 > $O/prof1.log 2>&1
rc=$?; echo "rc[prof1]=$rc"; [ $rc -eq 0 ] || exit $rc
python3 scripts/prof_summary.py $O/prof1 25 --tail-ms 200 --gaps 5 > $O/wave_summary_b1.txt 2>&1
rm -rf $O/prof1
exit 0
