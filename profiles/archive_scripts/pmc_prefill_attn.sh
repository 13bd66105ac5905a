#!/bin/bash
# rocprofv3 PMC passes (no trace domains) over the long-prompt prefill attention A/B
# (scripts/bench_prefill_attn.py at L = 8064): MFMA busy, VALU/LDS instruction mix, LDS bank
# conflicts and the wave-state split, per kernel. One pass per counter group, SIGKILL bound.
set -u
OUT=gpurun_out/pmc_pl
mkdir -p $OUT
ROOT=$(pwd)
export TMPDIR=/tmp
i=0
for pass in \
  "SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_MFMA SQ_INSTS_VALU GRBM_GUI_ACTIVE GRBM_COUNT" \
  "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS GRBM_GUI_ACTIVE"; do
  i=$((i + 1))
  echo "=== pass $i: $pass"
  cd /tmp
  timeout -s KILL 120 rocprofv3 --pmc $pass --output-format csv -d $ROOT/$OUT/pass$i -o pl \
    -- python $ROOT/scripts/bench_prefill_attn.py --lens ${PL_LENS:-8064} --rounds 1 \
       --out $ROOT/$OUT/bench_pass$i.json > $ROOT/$OUT/pass$i.log 2>&1
  rc=$?
  cd $ROOT
  echo "rc[pass$i]=$rc"; tail -3 $OUT/pass$i.log
  [ $rc -ne 0 ] && { echo "stopping"; exit $rc; }
done
python scripts/pmc_report.py $OUT/pass* > $OUT/pmc_report.txt 2>&1
grep -E "prefill_attn|kernel" $OUT/pmc_report.txt | head -20
