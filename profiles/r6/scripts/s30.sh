#!/bin/bash
# Session 30 (round 6): the decode-attention block-table window clamped to the table row
# instead of the context's last block (no dependency on context_lens) — attention / decode
# GPU tests, the Llama b512 wave, and the driver bench twice.
set -u
O=gpurun_out/r6s30
mkdir -p $O
: > $O/bench.jsonl
PT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 600 $PT tests/test_kernels_gpu.py tests/test_engine_gpu.py -k "attn or attention or decode or engine or paged" > $O/tests.log 2>&1
rc=$?; echo "rc[tests]=$rc"; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o wave -- python3 bench.py --steps 1 --warmup 1 > $O/prof.log 2>&1
rc=$?; echo "rc[prof]=$rc"; [ $rc -eq 0 ] || exit $rc
python3 scripts/prof_summary.py $O/prof 30 --tail-ms 800 --gaps 5 > $O/wave_summary.txt 2>&1
head -14 $O/wave_summary.txt
rm -rf $O/prof
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench_$i.log 2>&1
  rc=$?; echo "rc[bench_$i]=$rc"; [ $rc -eq 0 ] || exit $rc
  echo "{\"arm\": \"bench_$i\", \"bench\": $(grep -h '^{"metric"' $O/bench_$i.log)}" >> $O/bench.jsonl
  tail -1 $O/bench_$i.log
done
exit 0
