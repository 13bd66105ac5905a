# round 3, session AC: prefill-shape GEMMs (8-phase tile 22 with transposed epilogues) vs
# hipBLASLt, interleaved rounds, random operands, cold weights
set -o pipefail
mkdir -p gpurun_out/r3ac
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r3ac
echo "=== gemm8p $(date +%T)"; timeout -k 10 600 python -u scripts/bench_gemm8p.py --only prefill --tiles 22 --rounds 5 --out $O/prefill.json > $O/prefill.log 2>&1; echo "rc=$?"; tail -3 $O/prefill.log | cut -c1-400
timeout -k 10 300 python -u scripts/bench_gemm8p.py --only sq8192 --tiles 22 --rounds 3 --out $O/sq8192.json > $O/sq8192.log 2>&1; echo "rc=$?"; tail -1 $O/sq8192.log | cut -c1-400
echo "end $(date +%T)"
