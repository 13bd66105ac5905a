#!/usr/bin/env python3
"""Fixed cost of the decode GEMMs: each Llama-3-8B decode GEMM (M = 512) timed at its real K
and at one K-tile per workgroup (K = 64 x splits), same grid and same epilogue. The short-K
time is launch + prologue + epilogue (the fp32 split-K slab stores or the bf16 store), i.e.
what a deeper main loop cannot hide. Random bf16 operands, cold weights at the real K,
interleaved rounds in one process."""
import argparse
import json
import statistics
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from distributed_llm_inferencing_amd import ops  # noqa: E402
from distributed_llm_inferencing_amd.ops import gemm as G  # noqa: E402

# name, N, K, epi (0 bf16 / 2 silu), tile, splits
CASES = [
    ("qkv", 6144, 4096, 0, 23, 2),
    ("o", 4096, 4096, 0, 8, 4),
    ("gate_up", 28672, 4096, 2, 22, 1),
    ("down_t13", 4096, 14336, 0, 13, 8),
    ("down_t22", 4096, 14336, 0, 22, 8),
]


def launch(x, w, epi, tile, splits, ws, out):
    M, K = x.shape
    N = w.shape[0]
    c = None if splits > 1 else ops._p(out)
    ldc = N if splits > 1 else out.stride(0)
    ops._native_call("dli_gemm", ops._p(x), x.stride(0), ops._p(w), w.stride(-2), c, ldc,
                     M, N, K, epi, tile, splits, None, ops._p(ws), None, 1, ops._st())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--out", default="gpurun_out/epilogue.json")
    a = ap.parse_args()
    dev = torch.device("cuda")
    torch.manual_seed(0)
    M = 512
    res = []
    for name, N, K, epi, tile, splits in CASES:
        rec = {"name": name, "N": N, "tile": tile, "splits": splits}
        variants = {}
        for kk in (K, 64 * splits):
            w0 = (torch.rand(N, kk, device=dev) * 2 - 1).mul_(0.05).to(torch.bfloat16)
            ncp = max(1, min(8, -(-(600 << 20) // (w0.numel() * 2))))
            wl = [w0] + [w0.clone() for _ in range(ncp - 1)]
            x = (torch.rand(M, kk, device=dev) * 2 - 1).to(torch.bfloat16)
            ws = G.workspace(dev, splits * M * N * 4)
            out = torch.empty(M, N // 2 if epi == 2 else N, device=dev, dtype=torch.bfloat16)
            variants[kk] = (lambda x=x, wl=wl, ws=ws, out=out:
                            [launch(x, w, epi, tile, splits, ws, out) for w in wl], len(wl))
        times = {k: [] for k in variants}
        for _ in range(a.rounds):
            for k, (fn, n) in variants.items():
                times[k].append(ops.benchmark(fn, iters=4, warmup=1) * 1e3 / n)
        rec["us_full_K"] = statistics.median(times[K])
        rec["us_one_ktile"] = statistics.median(times[64 * splits])
        rec["tflops_full"] = 2.0 * M * N * K / (rec["us_full_K"] * 1e-6) / 1e12
        res.append(rec)
        print(json.dumps(rec), flush=True)
    Path(a.out).parent.mkdir(parents=True, exist_ok=True)
    Path(a.out).write_text(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
