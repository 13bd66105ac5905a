#!/usr/bin/env python3
"""Prefill-sized Llama-3-8B projections (M = --m rows, default 16384 = the headline wave's
512 prompts x 32 tokens) on each 256x256 plan the prefill autotune races, timed warm as
graph replays (the GEMMs are MFMA-bound). One JSON line per (shape, plan) with TF/s.

    python scripts/bench_prefill_gemm.py [--m 16384] [--shapes qkv,o,gate_up,down] [--tiles 22,45]
"""
import argparse
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

SHAPES = {"qkv": (6144, 4096, "none"), "o": (4096, 4096, "none"),
          "gate_up": (28672, 4096, "silu_mul"), "down": (4096, 14336, "none")}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=16384)
    ap.add_argument("--shapes", default="qkv,o,gate_up,down")
    ap.add_argument("--tiles", default="22,34,45")
    ap.add_argument("--splits", default="1")
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    from distributed_llm_inferencing_amd import ops
    from distributed_llm_inferencing_amd.ops import gemm as G
    dev = torch.device("cuda")
    torch.manual_seed(0)
    x = (torch.randn(a.m, 14336, device=dev) * 0.5).to(torch.bfloat16)
    for name in a.shapes.split(","):
        N, K, epi = SHAPES[name]
        w = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
        xa = x[:, :K].contiguous()
        flop = 2.0 * a.m * N * K
        for t in (int(v) for v in a.tiles.split(",")):
            for s in (int(v) for v in a.splits.split(",")):
                p = G.GemmPlan("dli", t, s)
                try:
                    ms = ops.benchmark(lambda p=p: ops._gemm_native(xa, w, epi, plan=p),
                                       iters=a.iters, warmup=2, graph=True)
                except Exception as e:  # noqa: BLE001
                    print(json.dumps({"shape": name, "tile": t, "splits": s, "error": str(e)}))
                    continue
                print(json.dumps({"shape": name, "M": a.m, "N": N, "K": K, "tile": t,
                                  "splits": s, "us": round(ms * 1e3, 1),
                                  "tflops": round(flop / (ms * 1e-3) / 1e12, 1)}), flush=True)
        del w, xa


if __name__ == "__main__":
    main()
