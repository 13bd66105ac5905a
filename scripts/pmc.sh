#!/bin/bash
# rocprofv3 PMC passes over one program, merged into a per-kernel counter table
# (scripts/pmc_report.py: MFMA busy %, GFLOP, L2->fabric and HBM bytes, LDS conflicts, wait /
# issue shares).
#
#   scripts/pmc.sh <out_dir> [program args...]
#
# The passes run from /tmp (rocprofv3's scratch), so give the program's paths absolute; the
# default program is "python3 <repo>/bench.py --steps 1 --warmup 1".
#
# One pass per counter group, each within the per-block slot limits (SQ 8, TCC 4 with
# FETCH_SIZE = 3 / WRITE_SIZE = 2, GRBM 2) and under its own SIGKILL timeout; counters the
# device does not list (rocprofv3 -L) are dropped from a pass before it runs. No trace domain
# is combined with --pmc, and the program itself follows `--` (no env / shell hop). Stops at
# the first non-zero exit.
set -u
OUT=${1:-gpurun_out/pmc}
shift || true
ROOT=$(pwd)
if [ $# -eq 0 ]; then set -- python3 "$ROOT/bench.py" --steps 1 --warmup 1; fi
mkdir -p "$OUT"
case "$OUT" in /*) ABS=$OUT ;; *) ABS=$ROOT/$OUT ;; esac
export TMPDIR=/tmp
timeout -k 10 90 rocprofv3 -L > "$ABS/counters.txt" 2>&1 || { echo "counter list failed"; exit 1; }
have() { grep -qw "$1" "$ABS/counters.txt"; }
i=0
for pass in \
  "SQ_WAVES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_MFMA SQ_INSTS_VALU GRBM_GUI_ACTIVE GRBM_COUNT" \
  "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS GRBM_GUI_ACTIVE" \
  "FETCH_SIZE GRBM_GUI_ACTIVE" \
  "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE" \
  "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum GRBM_GUI_ACTIVE"; do
  i=$((i + 1))
  sel=""
  for c in $pass; do
    if have "$c"; then sel="$sel $c"; else echo "pass $i: counter $c not listed, dropped"; fi
  done
  [ -z "$sel" ] && continue
  echo "=== pass $i:$sel"; date
  cd /tmp
  timeout -s KILL 300 rocprofv3 --pmc $sel --output-format csv -d "$ABS/pass$i" -o pmc \
    -- "$@" > "$ABS/pass$i.log" 2>&1
  rc=$?
  cd "$ROOT"
  echo "rc[pass$i]=$rc"; tail -3 "$ABS/pass$i.log"
  [ $rc -ne 0 ] && { echo "stopping"; exit $rc; }
done
python3 scripts/pmc_report.py "$ABS"/pass* > "$ABS/pmc_report.txt" 2>&1
# PMC_TAIL=N: a second table over each pass's last N dispatches only (a bench's timed wave,
# without the capture-time autotune probes)
if [ -n "${PMC_TAIL:-}" ]; then
  python3 scripts/pmc_report.py --tail "$PMC_TAIL" "$ABS"/pass* > "$ABS/pmc_report_tail.txt" 2>&1
fi
head -40 "$ABS/pmc_report.txt"
