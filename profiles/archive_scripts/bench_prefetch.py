"""Does pulling a weight into the Infinity Cache ahead of its GEMM pay at batch 1?

For each Llama-3-8B decode GEMM at M = 1 (plan: the heuristic, or --plan TILE,SPLITS):
  cold_us       the GEMM over a cold weight (copies cycled, > 1 GB in total)
  warm_us       the GEMM right after ops.prefetch() of the same weight
  after_mix_us  the GEMM after prefetch + one layer's gate/up + down GEMMs on other weights
                (does the prefetched weight survive ~350 MB of other streaming?)
  prefetch_gbs  ops.prefetch() throughput alone
Prints one JSON line per shape.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from distributed_llm_inferencing_amd import ops  # noqa: E402
from distributed_llm_inferencing_amd.ops import gemm as G  # noqa: E402

SHAPES = {"qkv": (6144, 4096, "none"), "o": (4096, 4096, "none"),
          "gate_up": (28672, 4096, "silu_mul"), "down": (4096, 14336, "none")}


def timed(fn, n):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn(0)
    torch.cuda.synchronize()
    s.record()
    for i in range(n):
        fn(i)
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / n          # us per iteration


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="qkv,o,gate_up,down")
    ap.add_argument("--wgs", type=int, default=256)
    ap.add_argument("--iters", type=int, default=48)
    a = ap.parse_args()
    dev = torch.device("cuda")
    torch.manual_seed(0)
    mix_gu = [torch.randn(28672, 4096, device=dev).to(torch.bfloat16) * 0.02 for _ in range(2)]
    mix_dn = [torch.randn(4096, 14336, device=dev).to(torch.bfloat16) * 0.02 for _ in range(2)]
    xg = torch.randn(1, 4096, device=dev).to(torch.bfloat16)
    xd = torch.randn(1, 14336, device=dev).to(torch.bfloat16)
    pg, pd = G.plan(1, 28672, 4096, "silu_mul"), G.plan(1, 4096, 14336, "none")

    def mix(i):
        ops._gemm_native(xg, mix_gu[i % 2], "silu_mul", plan=pg)
        ops._gemm_native(xd, mix_dn[i % 2], "none", plan=pd)
    for name in a.shapes.split(","):
        N, K, epi = SHAPES[name]
        nb = N * K * 2
        copies = max(4, min(24, (1 << 30) // nb + 1))
        ws = [torch.randn(N, K, device=dev).to(torch.bfloat16) * 0.02 for _ in range(copies)]
        x = torch.randn(1, K, device=dev).to(torch.bfloat16)
        p = G.plan(1, N, K, epi)

        def gemm(i):
            ops._gemm_native(x, ws[i % copies], epi, plan=p)

        def pf(i):
            ops.prefetch(ws[i % copies], max_wgs=a.wgs)
        cold = timed(gemm, a.iters)
        t_p = timed(pf, a.iters)
        t_pg = timed(lambda i: (pf(i), gemm(i)), a.iters)
        t_pm = timed(lambda i: (pf(i), mix(i)), a.iters)
        t_pmg = timed(lambda i: (pf(i), mix(i), gemm(i)), a.iters)
        print(json.dumps({"shape": name, "plan": [p.tile, p.splits], "MB": round(nb / 1e6, 1),
                          "cold_us": round(cold, 2), "warm_us": round(t_pg - t_p, 2),
                          "after_mix_us": round(t_pmg - t_pm, 2),
                          "prefetch_us": round(t_p, 2),
                          "prefetch_gbs": round(nb / t_p / 1e3, 1),
                          "cold_tbs": round(nb / cold / 1e6, 2)}), flush=True)
        del ws


if __name__ == "__main__":
    main()
