#!/bin/bash
# Session 20: GEMV tail steps batched (clamped loads, masked sums) + one b512 driver bench;
# session 19: the norm prologue split into issue / complete (row loads before the weight preload, counted wait);
# session 18: SiLU pairing tiles 58 / 59 (2 + 2 / 4 + 4 rows a workgroup);
# session 17: tiles 56 / 57 as general GEMV tiles and the prologue-aware autotune (QKV and gate/up timed with their deferred norm);
# batch-1 decode without split-K reduces (O / down GEMVs add into the residual,
# the next GEMV normalises in its prologue): kernel + engine tests, then batch-1 bench with
# the deferred norm on / off alternated on one box, and a rocprofv3 wave summary of batch 1.
set -u
O=gpurun_out/s20
mkdir -p $O
: > $O/bench.jsonl
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?;
         echo "rc[$name]=$rc"; tail -3 $O/$name.log; [ $rc -eq 0 ] || exit $rc; }
rec() { echo "{\"arm\": \"$1\", \"bench\": $(grep -h '^{"metric"' $O/$1.log)}" >> $O/bench.jsonl; }
step tests 600 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_kernels_gpu.py tests/test_engine_gpu.py -m gpu -k "gemv or residual or prologue or deferred or batch_invariant or graph_decode or loopback"
step b1_on_1 300 env DLI_DEFER_NORM=1 DLI_GEMM_AUTOTUNE_LOG=1 python3 bench.py --batch 1 --steps 8 --warmup 2
rec b1_on_1
grep "autotune\] M=1 " $O/b1_on_1.log > $O/autotune_picks_m1.txt || true
step b1_on_2 300 env DLI_DEFER_NORM=1 python3 bench.py --batch 1 --steps 8 --warmup 2
rec b1_on_2
step b512 300 python3 bench.py --gpus 1 --steps 20 --warmup 5
rec b512
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o wave -- python3 bench.py --batch 1 --steps 1 --warmup 1 > $O/prof.log 2>&1
rc=$?; echo "rc[prof]=$rc"; [ $rc -eq 0 ] || exit $rc
python3 scripts/prof_summary.py $O/prof 25 --tail-ms 230 --gaps 5 > $O/wave_summary.txt 2>&1
rm -rf $O/prof
exit 0
