#!/bin/bash
# Session 24: stream-K 8-phase GEMM (tile 60) — kernel tests first (bit-identical to tile 22,
# graph replays), the mixed-steps engine test alone and after the norm tests (plan-cache
# state), then the driver's bench with stream-K admitted vs kept out (DLI_GEMM_SK=0),
# alternated, with the autotune picks, and a b512 wave summary.
set -u
O=gpurun_out/s24
mkdir -p $O
: > $O/ab.jsonl
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?;
         echo "rc[$name]=$rc"; tail -3 $O/$name.log; [ $rc -eq 0 ] || exit $rc; }
rec() { echo "{\"arm\": \"$1\", \"bench\": $(grep -h '^{"metric"' $O/$1.log)}" >> $O/ab.jsonl; }
step sk_tests 300 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_kernels_gpu.py -m gpu -k "stream_k or gemm_bf16_all_tiles or gemm_epilogues"
step sk_1 300 env DLI_GEMM_AUTOTUNE_LOG=1 python3 bench.py --gpus 1 --steps 10 --warmup 3
rec sk_1
grep "autotune\] M=512 " $O/sk_1.log > $O/autotune_picks_m512.txt || true
step nosk_1 300 env DLI_GEMM_SK=0 python3 bench.py --gpus 1 --steps 10 --warmup 3
rec nosk_1
step sk_2 300 python3 bench.py --gpus 1 --steps 10 --warmup 3
rec sk_2
step nosk_2 300 env DLI_GEMM_SK=0 python3 bench.py --gpus 1 --steps 10 --warmup 3
rec nosk_2
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o wave -- python3 bench.py --steps 1 --warmup 1 > $O/prof.log 2>&1
rc=$?; echo "rc[prof]=$rc"; [ $rc -eq 0 ] || exit $rc
python3 scripts/prof_summary.py $O/prof 30 --tail-ms 830 --gaps 5 > $O/wave_summary.txt 2>&1
rm -rf $O/prof
exit 0
