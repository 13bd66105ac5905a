#!/bin/bash
# Same-box A/B of mixed prefill+decode steps end to end (scripts/serve_e2e.sh, config 2):
# arm "off" (DLI_MIXED_STEPS=0) then arm "on" (default), each a fresh master + worker.
# Usage: bash scripts/e2e_ab_mixed.sh [requests] [concurrency]
set -u
N=${1:-4096}; C=${2:-1024}
for arm in off on; do
  v=0; [ $arm = on ] && v=1
  DLI_MIXED_STEPS=$v timeout -k 10 560 bash scripts/serve_e2e.sh $N $C 512 > gpurun_out/e2e_$arm.log 2>&1
  rc=$?
  mkdir -p gpurun_out/e2e_mixed_$arm
  mv gpurun_out/e2e_*.json gpurun_out/e2e_mixed_$arm/ 2>/dev/null
  tail -3 gpurun_out/e2e_$arm.log
  echo "rc[$arm]=$rc"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
