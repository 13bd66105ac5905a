set -u
mkdir -p gpurun_out/s23b
timeout -k 10 300 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_engine_gpu.py -m gpu -k "mixed" > gpurun_out/s23b/mixed_only.log 2>&1; echo "rc_only=$?"; tail -2 gpurun_out/s23b/mixed_only.log
timeout -k 10 300 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_kernels_gpu.py tests/test_engine_gpu.py -m gpu -k "norm or mixed" > gpurun_out/s23b/norm_mixed.log 2>&1; echo "rc_nm=$?"; tail -2 gpurun_out/s23b/norm_mixed.log
