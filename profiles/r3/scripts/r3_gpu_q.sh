# round 3, session Q: transposed-accumulator GEMM epilogues (16-B / 8-B stores). Numerics,
# decode-projection landscape on this tree and on ./ab_base (HEAD before the change), and an
# interleaved bench A/B.
set -o pipefail
mkdir -p gpurun_out/r3q
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=$PWD/gpurun_out/r3q
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "rc[$name]=$rc"; tail -2 $O/$name.log | cut -c1-300; return $rc; }
run kern 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py -k "gemm or grouped or moe or linear" &&
run tiles_new 300 python -u scripts/bench_decode_tiles.py --shapes o,qkv,down,gate_up --top 4 &&
(cd ab_base && run tiles_base 300 python -u scripts/bench_decode_tiles.py --shapes o,qkv,down,gate_up --top 4) &&
run bench_new1 300 python -u bench.py --steps 3 --warmup 1 &&
(cd ab_base && run bench_base1 300 python -u bench.py --steps 3 --warmup 1) &&
run bench_new2 300 python -u bench.py --steps 3 --warmup 1 &&
(cd ab_base && run bench_base2 300 python -u bench.py --steps 3 --warmup 1)
echo "end $(date +%T)"
