#!/usr/bin/env python3
"""Per-op timings at the bench's decode shapes (Llama-3-8B, B=256, ctx 32..100), plus plain
device-copy rates to calibrate the memory-bound kernels against."""
import math
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from distributed_llm_inferencing_amd import ops  # noqa: E402
from distributed_llm_inferencing_amd.ops import reference as R  # noqa: E402


def main():
    dev = torch.device("cuda")
    B, hq, hkv, hd, bs, D, V = 256, 32, 8, 128, 16, 4096, 128256
    torch.manual_seed(0)
    lens = torch.randint(33, 100, (B,)).tolist()
    nblk = sum(-(-n // bs) for n in lens) + 16
    kc = (torch.randn(nblk, hkv, bs, hd, device=dev) * 0.5).to(torch.bfloat16)
    vc = (torch.randn(nblk, hkv, hd, bs, device=dev) * 0.5).to(torch.bfloat16)
    perm = torch.randperm(nblk).tolist()
    W = 32
    tables, o = [], 0
    for n in lens:
        nb = -(-n // bs)
        tables.append(perm[o:o + nb] + [0] * (W - nb))
        o += nb
    tables = torch.tensor(tables, device=dev, dtype=torch.int32)
    ctx = torch.tensor(lens, device=dev, dtype=torch.int32)
    qkv = torch.randn(B, (hq + 2 * hkv) * hd, device=dev).to(torch.bfloat16)
    res = {}
    kv_bytes = sum(lens) * hkv * hd * 2 * 2
    ms = ops.benchmark(lambda: ops.decode_attention(qkv, kc, vc, tables, ctx, 512, hq, hkv, hd,
                                                    1 / math.sqrt(hd)), iters=50)
    res["decode_attention"] = (ms * 1e3, kv_bytes / ms / 1e6)
    logits = torch.randn(B, V, device=dev) * 1.3
    t = torch.full((B,), 0.8, device=dev)
    k = torch.full((B,), 50, device=dev, dtype=torch.int32)
    p = torch.full((B,), 0.95, device=dev)
    s = torch.arange(B, device=dev, dtype=torch.int64)
    ms = ops.benchmark(lambda: ops.sample(logits, t, k, p, s), iters=30)
    res["sample_topk_topp"] = (ms * 1e3, B * V * 4 / ms / 1e6)
    x = torch.randn(B, D, device=dev).to(torch.bfloat16)
    r = torch.randn(B, D, device=dev).to(torch.bfloat16)
    w = torch.ones(D, device=dev, dtype=torch.bfloat16)
    ms = ops.benchmark(lambda: ops.add_rmsnorm(x, r, w, 1e-5), iters=50)
    res["add_rmsnorm"] = (ms * 1e3, 4 * B * D * 2 / ms / 1e6)
    # split-K reduce + residual add + RMSNorm alone, at the decode O/down shape (M=512, N=4096)
    from distributed_llm_inferencing_amd.ops import _native_call, _p, _st
    M2 = 512
    r2 = torch.randn(M2, D, device=dev).to(torch.bfloat16)
    o2 = torch.empty_like(r2)
    for spl in (2, 4, 8):
        ws = torch.randn(spl * M2 * D, device=dev)
        ms = ops.benchmark(lambda: _native_call("dli_splitk_add_rmsnorm", _p(o2), _p(r2), _p(ws),
                                                spl, M2, D, _p(w), 1e-5, _st()), iters=50)
        res[f"splitk{spl}_add_rmsnorm"] = (ms * 1e3, (spl * M2 * D * 4 + 3 * M2 * D * 2) / ms / 1e6)
    pos = ctx - 1
    slots = torch.arange(B, device=dev, dtype=torch.int32)
    cs = R.rope_cos_sin(2048, hd, 5e5, device=dev)
    ms = ops.benchmark(lambda: ops.rope_and_cache(qkv, pos, slots, cs, kc, vc, hq, hkv, hd),
                       iters=50)
    res["rope_cache"] = (ms * 1e3, qkv.numel() * 2 * 2 / ms / 1e6)
    # plain device copies for calibration (read + write bytes): a 1 GiB copy streams from HBM;
    # the 33 / 67 MB ones are the split-4 / split-8 slab sizes and, run back to back, stay
    # largely in the 256 MB Infinity Cache as the slabs a reduce reads right after its GEMM do
    for mb in (33, 67, 1024):
        n = mb * (1 << 20) // 4
        src, dst = torch.randn(n, device=dev), torch.empty(n, device=dev)
        ms = ops.benchmark(lambda: dst.copy_(src), iters=30)
        res[f"copy_{mb}MB"] = (ms * 1e3, 2 * n * 4 / ms / 1e6)
        del src, dst
    for kname, (us, gbs) in res.items():
        print(f"{kname:20s} {us:8.1f} us  {gbs:8.1f} GB/s")


if __name__ == "__main__":
    main()
