# round 3, session P (re-entry): full GPU tier + smoke + bench on the restored tree
set -o pipefail
mkdir -p gpurun_out/r3p
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r3p
run() { local name=$1 t=$2; shift 2; echo "=== $name $(date +%T)"; timeout -k 10 $t "$@" > $O/$name.log 2>&1; local rc=$?; echo "rc[$name]=$rc"; tail -2 $O/$name.log | cut -c1-400; return $rc; }
run pytest 1000 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread &&
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" &&
run bench 500 python -u bench.py --steps 5 --warmup 1
echo "end $(date +%T)"
