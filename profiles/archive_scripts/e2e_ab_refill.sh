#!/bin/bash
# Same-box A/B of the refill pacing interval end to end (scripts/serve_e2e.sh, config 2,
# mixed steps on): one fresh master + worker per arm, DLI_REFILL_INTERVAL_S = each argument.
# Usage: bash scripts/e2e_ab_refill.sh <requests> <concurrency> <interval>...
set -u
N=$1; C=$2; shift 2
for iv in "$@"; do
  DLI_REFILL_INTERVAL_S=$iv timeout -k 10 560 bash scripts/serve_e2e.sh $N $C 512 > gpurun_out/e2e_refill_$iv.log 2>&1
  rc=$?
  mkdir -p gpurun_out/e2e_refill_$iv
  mv gpurun_out/e2e_*.json gpurun_out/e2e_refill_$iv/ 2>/dev/null
  echo "refill=$iv rc=$rc $(python -c "import json;d=json.load(open('gpurun_out/e2e_refill_$iv/e2e_loadgen_c$C.json'));print({k:d.get(k) for k in ('requests_per_s','p50_latency_s','p99_latency_s','failed')})" 2>&1)"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
