# round 3: the full GPU test tier + smoke (what the driver runs at round end)
set -o pipefail
mkdir -p gpurun_out/r3full
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r3full
echo "=== pytest $(date +%T)"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "rc[pytest]=$rc"; tail -3 $O/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
echo "=== smoke $(date +%T)"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "rc[smoke]=$rc"; tail -3 $O/smoke.log
exit $rc
