#!/bin/bash
# rocprofv3 PMC passes over scripts/pmc_decode_ops.py (decode-layer kernels at batch 512).
# One pass per counter group, each within the per-block slot limits (SQ 8, TCC 4 with
# FETCH_SIZE=3 / WRITE_SIZE=2, GRBM 2) and under its own SIGKILL timeout; counters the
# device does not list (rocprofv3 -L) are dropped from a pass before it runs. No trace
# domains are combined with --pmc. Stops at the first non-zero exit.
set -u
OUT=gpurun_out/pmc
mkdir -p $OUT
ROOT=$(pwd)
export TMPDIR=/tmp
timeout -k 10 90 rocprofv3 -L > $OUT/counters.txt 2>&1 || { echo "counter list failed"; exit 1; }
timeout -k 10 180 python scripts/pmc_decode_ops.py --out $OUT/ops_timing.json > $OUT/timing.log 2>&1 \
  || { echo "timing run failed"; cat $OUT/timing.log; exit 1; }
cat $OUT/timing.log
have() { grep -qw "$1" $OUT/counters.txt; }
i=0
for pass in \
  "SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_MFMA SQ_INSTS_VALU GRBM_GUI_ACTIVE GRBM_COUNT" \
  "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS GRBM_GUI_ACTIVE" \
  "FETCH_SIZE GRBM_GUI_ACTIVE" \
  "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE" \
  "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum GRBM_GUI_ACTIVE" \
  "TCC_EA0_RDREQ_DRAM_sum TCC_BUBBLE_sum GRBM_GUI_ACTIVE"; do
  i=$((i + 1))
  sel=""
  for c in $pass; do
    if have "$c"; then sel="$sel $c"; else echo "pass $i: counter $c not listed, dropped"; fi
  done
  [ -z "$sel" ] && continue
  echo "=== pass $i:$sel"; date
  cd /tmp
  timeout -s KILL 120 rocprofv3 --pmc $sel --output-format csv -d $ROOT/$OUT/pass$i -o ops \
    -- python $ROOT/scripts/pmc_decode_ops.py --iters 3 --out $ROOT/$OUT/ops_pass$i.json \
    > $ROOT/$OUT/pass$i.log 2>&1
  rc=$?
  cd $ROOT
  echo "rc[pass$i]=$rc"; tail -5 $OUT/pass$i.log
  [ $rc -ne 0 ] && { echo "stopping"; break; }
done
python scripts/pmc_report.py $OUT/pass* > $OUT/pmc_report.txt 2>&1
cat $OUT/pmc_report.txt
