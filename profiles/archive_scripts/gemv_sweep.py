#!/usr/bin/env python3
"""Time every autotune candidate of the batch-1 decode GEMMs of Llama-3-8B (cold weights,
graph replay, each GEMM with its consumer exactly as ``ops.gemm.autotune`` times it) and
print one JSON line per (shape, plan). GPU only.

    python scripts/gemv_sweep.py [--m 1] [--out gpurun_out/gemv_sweep.jsonl]
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=1)
    ap.add_argument("--iters", type=int, default=8)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    from distributed_llm_inferencing_amd import ops
    from distributed_llm_inferencing_amd.ops import gemm as G
    dev = torch.device("cuda:0")
    M = a.m
    shapes = [("qkv", 6144, 4096, "none"), ("o", 4096, 4096, "splitk"),
              ("gate_up", 28672, 4096, "silu_mul"), ("down", 4096, 14336, "splitk"),
              ("lm_head", 128256, 4096, "f32")]
    out = open(a.out, "a") if a.out else None
    for name, N, K, epi in shapes:
        w0 = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
        n = max(2, min(16, -(-(1 << 30) // (w0.numel() * 2))))
        ws_ = [w0] + [w0.clone() for _ in range(n - 1)]
        x = (torch.randn(M, K, device=dev) * 0.5).to(torch.bfloat16)
        res = torch.zeros(M, N, dtype=torch.bfloat16, device=dev)
        nw = torch.ones(N, dtype=torch.bfloat16, device=dev)
        G.workspace(dev, 8 * M * N * 4)
        for p in G.candidate_plans(M, N, K, epi):
            def run(p=p):
                for w in ws_:
                    if epi == "splitk":
                        ops.linear_add_rmsnorm(x, w, res, nw, 1e-5, plan=p)
                    else:
                        ops._gemm_native(x, w, epi, plan=p)
            try:
                ms = ops.benchmark(run, iters=a.iters, warmup=1, graph=True) / len(ws_)
            except Exception as e:  # noqa: BLE001
                ms = None
            rec = {"shape": name, "M": M, "N": N, "K": K, "epi": epi, "tile": p.tile,
                   "splits": p.splits, "us": None if ms is None else round(ms * 1e3, 2),
                   "tb_s": None if not ms else round(N * K * 2 / (ms * 1e-3) / 1e12, 2)}
            line = json.dumps(rec)
            print(line, flush=True)
            if out:
                out.write(line + "\n")
        del ws_
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
