#!/usr/bin/env python3
"""Probe: can RCCL run 2 ranks on ONE GPU (same-device rehearsal of the pipeline's RCCL data
plane)? torchrun --nproc-per-node 2 scripts/nccl_probe.py. Prints one line per rank."""
import os
import sys

import torch
import torch.distributed as dist

rank = int(os.environ["RANK"])
torch.cuda.set_device(0)
dev = torch.device("cuda", 0)
dist.init_process_group("nccl", device_id=dev)
try:
    g = dist.new_group([0, 1])
    x = torch.full((4,), float(rank + 1), device=dev)
    if rank == 0:
        dist.isend(x, 1, group=g).wait()
        y = torch.empty(4, device=dev)
        dist.irecv(y, 1).wait()
    else:
        y = torch.empty(4, device=dev)
        dist.irecv(y, 0, group=g).wait()
        dist.isend(y * 10, 0).wait()
    torch.cuda.synchronize()
    print(f"rank {rank} OK {y.tolist()}", flush=True)
except Exception as e:  # noqa: BLE001
    print(f"rank {rank} FAILED {type(e).__name__}: {e}", flush=True)
    sys.exit(3)
finally:
    dist.destroy_process_group()
