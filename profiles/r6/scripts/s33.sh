#!/bin/bash
# Session 33 (round 6): prefill attention staging in named registers (the compiler had promoted
# the uint4[PER] staging arrays to LDS) on top of the 72-dword K rows — same steps as s32.
set -u
O=gpurun_out/r6s33
mkdir -p $O
: > $O/bench.jsonl
PT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 600 $PT tests/test_kernels_gpu.py tests/test_engine_gpu.py -k "prefill or attn or attention or chunk or engine" > $O/tests.log 2>&1
rc=$?; echo "rc[tests]=$rc"; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o wave -- python3 $R/bench.py --steps 1 --warmup 1 > $R/$O/prof.log 2>&1
rc=$?; echo "rc[prof]=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS GRBM_GUI_ACTIVE --kernel-include-regex prefill_attn --output-format csv -d $R/$O/pmc -o pmc -- python3 $R/bench.py --steps 1 --warmup 1 > $R/$O/pmc.log 2>&1
rc=$?; echo "rc[pmc]=$rc"; [ $rc -eq 0 ] || exit $rc
cd $R
python3 scripts/prof_summary.py $O/prof 30 --tail-ms 800 --gaps 5 > $O/wave_summary.txt 2>&1
head -16 $O/wave_summary.txt
python3 scripts/pmc_report.py $O/pmc > $O/pmc_report.txt 2>&1
head -6 $O/pmc_report.txt
rm -rf $O/prof $O/pmc
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench_$i.log 2>&1
  rc=$?; echo "rc[bench_$i]=$rc"; [ $rc -eq 0 ] || exit $rc
  echo "{\"arm\": \"bench_$i\", \"bench\": $(grep -h '^{"metric"' $O/bench_$i.log)}" >> $O/bench.jsonl
  tail -1 $O/bench_$i.log | cut -c1-200
done
exit 0
