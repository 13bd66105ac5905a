#!/usr/bin/env python3
"""Every autotune candidate plan for the Llama-3-8B decode projections at one batch size,
timed the way the autotuner times them (cold weights: a different weight copy per call,
together larger than the Infinity Cache; split-K plans with their slab reduction through the
fused add+RMSNorm consumer for "splitk" shapes). Prints one JSON line per (shape, plan),
sorted by time, so the whole landscape is visible rather than only the winner.

    python scripts/bench_decode_tiles.py [--m 512] [--shapes o,qkv]
"""
import argparse
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

SHAPES = {"qkv": (6144, 4096, "splitk"), "o": (4096, 4096, "splitk"),
          "gate_up": (28672, 4096, "silu_mul"), "down": (4096, 14336, "splitk"),
          "head": (128256, 4096, "f32")}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=512)
    ap.add_argument("--shapes", default="o,qkv")
    ap.add_argument("--iters", type=int, default=6)
    ap.add_argument("--slab-store", type=int, default=0,
                    help="split-K partial stores: 0 plain, 1 nt, 2 sc1, 3 sc0 sc1")
    ap.add_argument("--top", type=int, default=0, help="print only the N fastest plans")
    a = ap.parse_args()
    from distributed_llm_inferencing_amd import ops
    from distributed_llm_inferencing_amd.ops import _native as NT
    NT.require_native().dli_gemm_set_slab_store(a.slab_store)
    from distributed_llm_inferencing_amd.ops import gemm as G
    dev = torch.device("cuda")
    for name in a.shapes.split(","):
        N, K, epi = SHAPES[name]
        w0 = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
        n_copies = max(2, min(16, -(-(1 << 30) // (w0.numel() * 2))))
        ws_ = [w0] + [w0.clone() for _ in range(n_copies - 1)]
        x = (torch.randn(a.m, K, device=dev) * 0.5).to(torch.bfloat16)
        res = torch.zeros(a.m, N, dtype=torch.bfloat16, device=dev)
        nw = torch.ones(N, dtype=torch.bfloat16, device=dev)
        rows = []
        for p in G.candidate_plans(a.m, N, K, epi):
            def run(p=p):
                for w in ws_:
                    if epi == "splitk":
                        ops.linear_add_rmsnorm(x, w, res, nw, 1e-5, plan=p)
                    else:
                        ops._gemm_native(x, w, epi, plan=p)
            try:
                ms = ops.benchmark(run, iters=a.iters, warmup=1) / len(ws_)
            except Exception as e:  # noqa: BLE001
                rows.append({"shape": name, "tile": p.tile, "splits": p.splits,
                             "error": str(e)[:80]})
                continue
            rows.append({"shape": name, "M": a.m, "slab_store": a.slab_store, "tile": p.tile,
                         "bm_bn": G.TILES.get(p.tile, ("gemv", G.GEMV_TILES.get(p.tile))),
                         "splits": p.splits, "us": round(ms * 1e3, 2),
                         "tflops": round(2 * a.m * N * K / (ms * 1e-3) / 1e12, 1)})
        for r in sorted(rows, key=lambda r: r.get("us", 1e9))[:a.top or None]:
            print(json.dumps(r), flush=True)
        del ws_


if __name__ == "__main__":
    main()
