#!/usr/bin/env python3
"""Mid-sized prefill GEMMs (serving refills / mixed steps, M ~ 1-2k rows) on the 8-phase tile:
no split vs the split-K the planner now picks, each timed WITH its consumer (fused split-K
reduce + residual/RMSNorm or RoPE stand-in; the unsplit arm runs the bf16 GEMM + the
separate add+RMSNorm pass), cold weights (16 copies > Infinity Cache)."""
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from distributed_llm_inferencing_amd import ops  # noqa: E402
from distributed_llm_inferencing_amd.ops import gemm as G  # noqa: E402


def main():
    dev = torch.device("cuda")
    torch.manual_seed(0)
    for M in (1024, 1200, 1536, 2048):
        for N, K in ((6144, 4096), (4096, 4096), (4096, 14336)):
            ws = [(torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16) for _ in range(8)]
            x = (torch.randn(M, K, device=dev) * 0.5).to(torch.bfloat16)
            res = torch.zeros(M, N, dtype=torch.bfloat16, device=dev)
            nw = torch.ones(N, dtype=torch.bfloat16, device=dev)
            pick = G._heuristic(M, N, K, "splitk")
            row = {"M": M, "N": N, "K": K, "pick_splits": pick.splits}
            for s in sorted({1, pick.splits}):
                p = G.GemmPlan("dli", 22, s)
                ms = ops.benchmark(lambda: [ops.linear_add_rmsnorm(x, w, res, nw, 1e-5, plan=p)
                                            for w in ws], iters=5, warmup=1) / len(ws)
                row[f"us_split{s}"] = round(ms * 1e3, 1)
            print(json.dumps(row), flush=True)
            del ws


if __name__ == "__main__":
    main()
