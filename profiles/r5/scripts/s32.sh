#!/bin/bash
# Session 32: the norm-prologue GEMVs with the prologue width as a template parameter (the
# unused 4-vector branch had set 196 VGPRs at MB = 4): GEMV + engine tests, batch 4 and
# batch 1 benches, a batch-4 wave summary.
set -u
O=gpurun_out/s32
mkdir -p $O
: > $O/bench.jsonl
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?;
         echo "rc[$name]=$rc"; tail -2 $O/$name.log; [ $rc -eq 0 ] || exit $rc; }
rec() { echo "{\"arm\": \"$1\", \"bench\": $(grep -h '^{"metric"' $O/$1.log)}" >> $O/bench.jsonl; }
step tests 600 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_kernels_gpu.py tests/test_engine_gpu.py -m gpu -k "gemv or prologue or residual or deferred or batch_invariant or graph_decode or loopback"
step b4 240 env DLI_GEMM_AUTOTUNE_LOG=1 python3 bench.py --batch 4 --steps 4 --warmup 1
rec b4
grep "autotune\] M=4 " $O/b4.log > $O/autotune_picks_m4.txt || true
step b1 240 python3 bench.py --batch 1 --steps 8 --warmup 2
rec b1
step b4_2 240 python3 bench.py --batch 4 --steps 4 --warmup 1
rec b4_2
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof4 -o wave -- python3 bench.py --batch 4 --steps 1 --warmup 1 > $O/prof4.log 2>&1
rc=$?; echo "rc[prof4]=$rc"; [ $rc -eq 0 ] || exit $rc
python3 scripts/prof_summary.py $O/prof4 16 --tail-ms 260 > $O/wave_summary_b4.txt 2>&1
rm -rf $O/prof4
exit 0
