#!/bin/bash
# rocprofv3 counter passes over scripts/pmc_gemm.py (prefill GEMMs: 8-phase tile 22,
# two-barrier 4-wave tile 45, hipBLASLt). One pass per counter group within the per-block
# slot limits, each under its own SIGKILL timeout; no trace domains with --pmc.
set -u
OUT=${1:-gpurun_out/pmc_gemm}
mkdir -p $OUT
ROOT=$(pwd)
export TMPDIR=/tmp
timeout -k 10 90 rocprofv3 -L > $OUT/counters.txt 2>&1 || { echo "counter list failed"; exit 1; }
have() { grep -qw "$1" $OUT/counters.txt; }
i=0
for pass in \
  "SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_MFMA SQ_INSTS_VALU GRBM_GUI_ACTIVE GRBM_COUNT" \
  "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS GRBM_GUI_ACTIVE" \
  "FETCH_SIZE GRBM_GUI_ACTIVE"; do
  i=$((i + 1))
  sel=""
  for c in $pass; do
    if have "$c"; then sel="$sel $c"; else echo "pass $i: counter $c not listed, dropped"; fi
  done
  [ -z "$sel" ] && continue
  echo "=== pass $i:$sel"; date
  cd /tmp
  timeout -s KILL 120 rocprofv3 --pmc $sel --output-format csv -d $ROOT/$OUT/pass$i -o gemm \
    -- python3 $ROOT/scripts/pmc_gemm.py --iters 3 > $ROOT/$OUT/pass$i.log 2>&1
  rc=$?
  cd $ROOT
  echo "rc[pass$i]=$rc"; tail -2 $OUT/pass$i.log
  [ $rc -ne 0 ] && { echo "stopping"; exit $rc; }
done
python3 scripts/pmc_report.py $OUT/pass* > $OUT/report.txt && cat $OUT/report.txt | head -20
