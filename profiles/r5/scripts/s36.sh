#!/bin/bash
# Session 36: the driver's exact GPU-tier form (one pytest invocation, -q, every GPU test).
set -u
O=gpurun_out/s36
mkdir -p $O
timeout -k 10 1000 python -m pytest tests/ -x -q -m gpu > $O/tier.log 2>&1; rc=$?
echo "rc[tier]=$rc"; tail -3 $O/tier.log
exit $rc
