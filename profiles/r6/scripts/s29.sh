#!/bin/bash
# Session 29 (round 6): the driver's torchrun form of the multi-GPU bench (one rank per
# process under torch.distributed.run, 127.0.0.1 rendezvous), both ranks on the one GPU of
# this box (DLI_SAME_DEVICE=1), pp2.
set -u
O=gpurun_out/r6s29
mkdir -p $O
export DLI_SAME_DEVICE=1 DLI_GEMM_AUTOTUNE=0
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 > $O/torchrun_pp2.log 2>&1
rc=$?; echo "rc[torchrun_pp2]=$rc"; grep -h '^{"metric"' $O/torchrun_pp2.log | tail -1; tail -3 $O/torchrun_pp2.log
exit $rc
