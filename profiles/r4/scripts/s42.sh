#!/bin/bash
# round 4, session 42: rocprofv3 kernel summary of the batch-1 wave at HEAD (tile 29 gate/up)
set -o pipefail
R=$(pwd); O=$R/gpurun_out/r4s42; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p -o run -- python3 $R/bench.py --batch 1 --steps 3 --warmup 1 > $O/prof_b1.log 2>&1
rc=$?; echo "rc[prof]=$rc"; [ $rc -eq 0 ] || exit $rc
cd $R
python3 scripts/prof_summary.py $O/p 30 --tail-ms 900 > $O/b1_wave.txt && rm -rf $O/p
grep -h '"value"' $O/prof_b1.log | cut -c90-260
head -16 $O/b1_wave.txt
echo "end $(date +%T)"
