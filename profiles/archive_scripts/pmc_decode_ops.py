#!/usr/bin/env python3
"""Short driver for rocprofv3 --pmc passes: the hot kernels of one Llama-3-8B decode layer at
batch 512 (the bench config), each run ``--iters`` times with the plans the capture-time
autotuner picks on MI355X (profiles/r1_s4/autotune_with_consumer.txt), plus the LM head and
the sampler. No hipGraphs, so every dispatch is a separate counter record; prints the analytic
FLOPs / bytes per kernel so scripts/pmc_report.py can turn counters into utilisation."""
import argparse
import json
import math
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from distributed_llm_inferencing_amd import ops  # noqa: E402
from distributed_llm_inferencing_amd.ops import gemm as G  # noqa: E402
from distributed_llm_inferencing_amd.ops import reference as R  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--B", type=int, default=512)
    ap.add_argument("--out", default="gpurun_out/pmc/ops.json")
    a = ap.parse_args()
    dev = torch.device("cuda")
    torch.manual_seed(0)
    B, D, F, hq, hkv, hd, V, bs = a.B, 4096, 14336, 32, 8, 128, 128256, 16
    nqkv = (hq + 2 * hkv) * hd
    w = {n: (torch.randn(s, device=dev) * 0.02).to(torch.bfloat16) for n, s in
         (("qkv", (nqkv, D)), ("o", (D, D)), ("gu", (2 * F, D)), ("down", (D, F)),
          ("head", (V, D)))}
    x = torch.randn(B, D, device=dev).to(torch.bfloat16)
    h = torch.randn(B, F, device=dev).to(torch.bfloat16)
    res = torch.randn(B, D, device=dev).to(torch.bfloat16)
    nw = torch.ones(D, device=dev, dtype=torch.bfloat16)
    # plans the in-situ autotuner picks at M=512 (with their fused reduces; round 4:
    # profiles/r4/prof/llama_b512_head.wave.txt)
    G.set_plan(B, nqkv, D, "splitk", G.GemmPlan("dli", 23, 2))
    G.set_plan(B, D, D, "splitk", G.GemmPlan("dli", 16, 4))
    G.set_plan(B, 2 * F, D, "silu_mul", G.GemmPlan("dli", 22, 1))
    G.set_plan(B, D, F, "splitk", G.GemmPlan("dli", 22, 8))
    G.set_plan(B, V, D, "f32", G.GemmPlan("dli", 22, 1))

    lens = torch.randint(33, 100, (B,)).tolist()
    nblk = sum(-(-n // bs) for n in lens) + 16
    kc = (torch.randn(nblk, hkv, bs, hd, device=dev) * 0.5).to(torch.bfloat16)
    vc = (torch.randn(nblk, hkv, hd, bs, device=dev) * 0.5).to(torch.bfloat16)
    perm = torch.randperm(nblk).tolist()
    Wt, tables, o = 8, [], 0
    for n in lens:
        nb = -(-n // bs)
        tables.append(perm[o:o + nb] + [0] * (Wt - nb))
        o += nb
    tables = torch.tensor(tables, device=dev, dtype=torch.int32)
    ctx = torch.tensor(lens, device=dev, dtype=torch.int32)
    pos = ctx - 1
    slots = torch.tensor([tables[i, (lens[i] - 1) // bs].item() * bs + (lens[i] - 1) % bs
                          for i in range(B)], device=dev, dtype=torch.int32)
    cs = R.rope_cos_sin(2048, hd, 5e5, device=dev)
    t = torch.full((B,), 0.8, device=dev)
    k = torch.full((B,), 50, device=dev, dtype=torch.int32)
    p = torch.full((B,), 0.95, device=dev)
    seeds = torch.arange(B, device=dev, dtype=torch.int64)
    kv_bytes = sum(lens) * hkv * hd * 2 * 2

    def gemm_cost(N, K, splits=1, out_b=2):
        return 2 * B * N * K, 2 * (N * K + B * K) + (splits * 4 if splits > 1 else out_b) * B * N

    steps = {
        "qkv+rope_cache": (lambda: ops.linear_rope_cache(x, w["qkv"], pos, slots, cs, kc, vc,
                                                         hq, hkv, hd), gemm_cost(nqkv, D, 2)),
        "decode_attention": (lambda: ops.decode_attention(qkv0, kc, vc, tables, ctx, Wt * bs,
                                                          hq, hkv, hd, 1 / math.sqrt(hd)),
                             (4 * hq * hd * sum(lens), kv_bytes)),
        "o+add_rmsnorm": (lambda: ops.linear_add_rmsnorm(x, w["o"], res, nw, 1e-5),
                          gemm_cost(D, D, 4)),
        "gate_up+silu": (lambda: ops.linear(x, w["gu"], epi="silu_mul"), gemm_cost(2 * F, D)),
        "down+add_rmsnorm": (lambda: ops.linear_add_rmsnorm(h, w["down"], res, nw, 1e-5),
                             gemm_cost(D, F, 8)),
        "lm_head": (lambda: ops.linear(x, w["head"], epi="f32"), gemm_cost(V, D, 1, 4)),
        "sample": (lambda: ops.sample(logits, t, k, p, seeds), (0, B * V * 4)),
    }
    qkv0 = torch.randn(B, nqkv, device=dev).to(torch.bfloat16)
    logits = (torch.randn(B, V, device=dev) * 1.3)
    out = {}
    for name, (fn, (flops, byts)) in steps.items():
        fn()
        torch.cuda.synchronize()
        ms = ops.benchmark(fn, iters=a.iters, warmup=1)
        out[name] = {"us": ms * 1e3, "flops": flops, "bytes": byts,
                     "tflops": flops / ms / 1e9, "gbps": byts / ms / 1e6}
        print(json.dumps({name: out[name]}), flush=True)
    Path(a.out).parent.mkdir(parents=True, exist_ok=True)
    Path(a.out).write_text(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
