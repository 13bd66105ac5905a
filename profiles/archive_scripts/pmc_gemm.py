#!/usr/bin/env python3
"""Prefill-sized projection GEMMs (Llama-3-8B at 16,384 tokens: QKV and down) on our 8-phase
tile (22), the two-barrier 4-wave tile (45) and hipBLASLt (torch.matmul), a few calls each —
the workload of scripts/pmc_gemm.sh's counter passes (kernels are told apart by name)."""
import argparse
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=3)
    a = ap.parse_args()
    from distributed_llm_inferencing_amd import ops
    from distributed_llm_inferencing_amd.ops import gemm as G
    dev = torch.device("cuda")
    torch.manual_seed(0)
    for M, N, K in ((16384, 6144, 4096), (16384, 4096, 14336)):
        x = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
        w = (torch.rand(N, K, device=dev) * 2 - 1).mul_(0.05).to(torch.bfloat16)
        for _ in range(a.iters):
            for tile in (22, 45):
                ops._gemm_native(x, w, "none", plan=G.GemmPlan("dli", tile, 1))
            torch.matmul(x, w.t())
        torch.cuda.synchronize()
        print(f"M={M} N={N} K={K} done", flush=True)


if __name__ == "__main__":
    main()
