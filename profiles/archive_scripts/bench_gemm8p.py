#!/usr/bin/env python3
"""A/B of the 8-phase ping-pong 256x256 GEMM (tile 22) against the 2-stage 8-wave 256x256
tile (13) and hipBLASLt on the Llama-3-8B decode / prefill shapes. Random bf16 operands
(cdna_hip_programming.md §5.4 rule 25), cold weights (one copy per call, copies > 256 MB
Infinity Cache), interleaved rounds in one process (rule 24). Checks every dli result
against an fp32 torch reference first."""
import argparse
import json
import statistics
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from distributed_llm_inferencing_amd import ops  # noqa: E402
from distributed_llm_inferencing_amd.ops import gemm as G  # noqa: E402

# name, M, N, K, epi, splits for the dli tiles
CASES = [
    ("gate_up_silu_b512", 512, 28672, 4096, "silu_mul", 1),
    ("gate_up_b256", 256, 28672, 4096, "silu_mul", 1),
    ("down_b512_s8", 512, 4096, 14336, "splitk", 8),
    ("down_b512_s4", 512, 4096, 14336, "splitk", 4),
    ("qkv_b512_s4", 512, 6144, 4096, "splitk", 4),
    ("o_b512_s4", 512, 4096, 4096, "splitk", 4),
    ("lm_head_b512", 512, 128256, 4096, "f32", 1),
    ("sq4096", 4096, 4096, 4096, "none", 1),
    ("prefill_gate_up", 16384, 28672, 4096, "silu_mul", 1),
    ("prefill_qkv", 16384, 6144, 4096, "none", 1),
    ("prefill_down", 16384, 4096, 14336, "none", 1),
    ("odd_M300", 300, 4096, 4096, "none", 1),
    ("sq8192", 8192, 8192, 8192, "none", 1),
]


def ref(x, w, epi):
    y = x.float() @ w.float().t()
    if epi == "silu_mul":
        N = y.shape[1]
        y = y.view(y.shape[0], N // 32, 2, 16)
        y = (torch.nn.functional.silu(y[:, :, 0]) * y[:, :, 1]).reshape(y.shape[0], N // 2)
    return y


def run_dli(x, w, epi, tile, splits):
    M, K = x.shape
    N = w.shape[0]
    if epi == "splitk":        # slabs only (the fused reduce consumes them in the model)
        ws = G.workspace(x.device, splits * M * N * 4)
        ops._native_call("dli_gemm", ops._p(x), x.stride(0), ops._p(w), w.stride(-2), None, N,
                         M, N, K, 0, tile, splits, None, ops._p(ws), None, 1, ops._st())
        return ws[: splits * M * N * 4].view(torch.float32).view(splits, M, N).sum(0)
    return ops._gemm_native(x, w, epi, plan=G.GemmPlan("dli", tile, splits))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--iters", type=int, default=4)
    ap.add_argument("--out", default="gpurun_out/gemm8p.json")
    ap.add_argument("--only", default="")
    ap.add_argument("--tiles", default="13,22,26")
    a = ap.parse_args()
    dev = torch.device("cuda")
    torch.manual_seed(0)
    res = []
    for name, M, N, K, epi, splits in CASES:
        if a.only and a.only not in name:
            continue
        w0 = (torch.rand(N, K, device=dev) * 2 - 1).mul_(0.05).to(torch.bfloat16)
        ncp = max(1, min(8, -(-(600 << 20) // (w0.numel() * 2))))
        wl = [w0] + [w0.clone() for _ in range(ncp - 1)]
        x = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
        r = ref(x, w0, epi)
        scale = r.abs().max().item() + 1e-6
        errs = {}
        tiles = [int(t) for t in a.tiles.split(",")]
        for tile in tiles:
            try:
                y = run_dli(x, w0, epi, tile, splits)
                torch.cuda.synchronize()
                errs[tile] = (y.float() - r).abs().max().item() / scale
            except Exception as e:  # noqa: BLE001
                errs[tile] = f"error: {e}"
        variants = {t: (lambda t=t: [run_dli(x, w, epi, t, splits) for w in wl])
                    for t in tiles if isinstance(errs[t], float)}
        if epi in ("none", "splitk"):
            variants["blas"] = lambda: [torch.matmul(x, w.t()) for w in wl]
        times = {k: [] for k in variants}
        for _ in range(a.rounds):
            for k, fn in variants.items():
                times[k].append(ops.benchmark(fn, iters=a.iters, warmup=1) * 1e3 / len(wl))
        flops = 2.0 * M * N * K
        rec = {"name": name, "M": M, "N": N, "K": K, "epi": epi, "splits": splits,
               "rel_err": {str(k): v for k, v in errs.items()},
               "us_median": {str(k): statistics.median(v) for k, v in times.items()},
               "us_min": {str(k): min(v) for k, v in times.items()}}
        rec["tflops"] = {k: flops / (u * 1e-6) / 1e12 for k, u in rec["us_median"].items()}
        res.append(rec)
        print(json.dumps(rec), flush=True)
    Path(a.out).parent.mkdir(parents=True, exist_ok=True)
    Path(a.out).write_text(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
