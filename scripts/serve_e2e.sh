#!/bin/bash
# End-to-end serving on one MI355X through the public API (BASELINE.json config 2: master
# dispatch -> one Llama-3-8B worker): master (Flask, sqlite store, request queue,
# dispatcher pool) + one GPU worker (continuous batching over HTTP requests) + the load
# generator submitting form-encoded requests exactly as the reference UI does and polling
# /api/inference/status/<id>/. Reference request shape: max_length 100 incl. the prompt,
# T=0.8 / top-k 50 / top-p 0.95 (the dispatcher's defaults, views.py:351).
#
# Phases: warm-up (graphs already captured by --preload), closed loop at concurrency C
# (N requests), then concurrency 1 (latency of a lone request through every hop).
# Usage: bash scripts/serve_e2e.sh [requests] [concurrency] [max_batch] [server]
set -u
N=${1:-1024}; C=${2:-512}; B=${3:-512}; SRV=${4:-aiohttp}
mkdir -p gpurun_out/logs
export MASTER_DB=/tmp/dli_e2e_$$.sqlite3 DLI_LOG_DIR=gpurun_out/logs DISPATCH_WORKERS=$C
export HSA_ENABLE_IPC_MODE_LEGACY=0
python -m distributed_llm_inferencing_amd.cli serve-master --port 8000 --server $SRV \
    > gpurun_out/e2e_master.log 2>&1 &
MPID=$!
python -m distributed_llm_inferencing_amd.cli serve-worker --port 5000 --gpu 0 --max-batch $B --server $SRV \
    --preload llama3-8b > gpurun_out/e2e_worker.log 2>&1 &
WPID=$!
cpu() { awk '{print $14 + $15}' /proc/$1/stat; }   # utime + stime, clock ticks
ok=0
for i in $(seq 1 600); do
  if curl -sf http://127.0.0.1:5000/health | grep -q llama3-8b; then ok=1; break; fi
  if ! kill -0 $WPID 2>/dev/null; then break; fi
  sleep 1
done
rc=1
if [ $ok = 1 ]; then
  curl -s -X POST -d hostname=gpu0 -d ip_address=127.0.0.1 -d port=5000 \
      http://127.0.0.1:8000/api/nodes/add/ > gpurun_out/e2e_addnode.json
  LG="python -m distributed_llm_inferencing_amd.loadgen --master http://127.0.0.1:8000 --model llama3-8b --prompt-words 5"
  # warm-up wave (same shape)
  timeout -k 10 600 $LG --requests $C --concurrency $C --seed 99 > gpurun_out/e2e_warmup.json && \
  curl -s http://127.0.0.1:5000/metrics > gpurun_out/e2e_metrics_before.json && \
  cpu0="$(cpu $MPID) $(cpu $WPID) $(date +%s.%N)" && \
  timeout -k 10 900 $LG --requests $N --concurrency $C > gpurun_out/e2e_loadgen_c$C.json && \
  cpu1="$(cpu $MPID) $(cpu $WPID) $(date +%s.%N)" && \
  python -c "import json,sys,os; a=[float(x) for x in sys.argv[1].split()]; b=[float(x) for x in sys.argv[2].split()]; hz=os.sysconf('SC_CLK_TCK'); w=b[2]-a[2]; print(json.dumps({'wall_s': round(w,3), 'master_cores_busy': round((b[0]-a[0])/hz/w,3), 'worker_cores_busy': round((b[1]-a[1])/hz/w,3)}))" "$cpu0" "$cpu1" > gpurun_out/e2e_cpu.json && \
  curl -s http://127.0.0.1:5000/metrics > gpurun_out/e2e_metrics_after.json && \
  timeout -k 10 600 $LG --requests 16 --concurrency 1 --poll 0.01 > gpurun_out/e2e_loadgen_c1.json
  rc=$?
  cat gpurun_out/e2e_loadgen_c$C.json gpurun_out/e2e_loadgen_c1.json
  curl -s http://127.0.0.1:8000/metrics > gpurun_out/e2e_master_metrics.json
else
  echo "worker did not become healthy"; tail -20 gpurun_out/e2e_worker.log
fi
kill $WPID $MPID 2>/dev/null
wait
rm -f $MASTER_DB
exit $rc
