#!/usr/bin/env python3
"""Decode attention at batch 512 (Llama-3-8B heads: 32 q / 8 kv x 128) against context
length: the fused kernel the decode graph runs (QKV split-K fp16 slabs reduced, RoPE, k/v
cache write and attention in one launch), and the unfused plain / pipelined attention kernels
(timed apart from the separate RoPE + cache-write kernel). Times are per call from graph replays of 16 calls each; the KV
bytes read per call give the achieved bandwidth, and the slope / intercept of time against
context split the per-token (streaming) cost from the fixed (prologue, launch) cost.

    python scripts/attn_probe.py [--batch 64,512] [--ctx 1,33,66,100,200,400]
"""
import argparse
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", default="512")
    ap.add_argument("--ctx", default="1,33,66,100,200,400")
    ap.add_argument("--reps", type=int, default=7)
    a = ap.parse_args()
    from distributed_llm_inferencing_amd import ops
    dev = torch.device("cuda")
    hq, hkv, hd, bs = 32, 8, 128, 16
    R = 16
    N = (hq + 2 * hkv) * hd
    scale = hd ** -0.5
    cos_sin = torch.randn(4096, hd, device=dev)
    for B, ctx in [(int(b), int(c)) for b in a.batch.split(",") for c in a.ctx.split(",")]:
        nblk_seq = -(-ctx // bs)
        nblk = B * nblk_seq + 8
        kc = (torch.randn(nblk, hkv, bs, hd, device=dev) * 0.5).to(torch.bfloat16)
        vc = (torch.randn(nblk, hkv, bs, hd, device=dev) * 0.5).to(torch.bfloat16)
        perm = torch.randperm(nblk - 8, device=dev).to(torch.int32)
        bt = perm[:B * nblk_seq].view(B, nblk_seq).contiguous()
        cl = torch.full((B,), ctx, dtype=torch.int32, device=dev)
        pos = cl - 1
        slot = (bt[:, (ctx - 1) // bs] * bs + (ctx - 1) % bs).to(torch.int32)
        slabs = (torch.randn(2, B, N, device=dev) * 0.02).to(torch.float16)
        qkv = (torch.randn(B, N, device=dev) * 0.5).to(torch.bfloat16)
        out = torch.empty(B, hq * hd, dtype=torch.bfloat16, device=dev)
        kv_mb = B * hkv * ctx * 2 * hd * 2 / 1e6

        def fused():
            ops._native_call("dli_decode_attention_fused", ops._p(out), ops._p(slabs), 2,
                             ops._p(pos), ops._p(slot), ops._p(cos_sin), ops._p(kc), ops._p(vc),
                             ops._p(bt), bt.stride(0), ops._p(cl), B, hq, hkv, hd, bs, scale, 1,
                             ops._st())

        def rope():
            ops.rope_and_cache(qkv, pos, slot, cos_sin, kc, vc, hq, hkv, hd)

        def attn():
            ops.decode_attention(qkv, kc, vc, bt, cl, ctx, hq, hkv, hd, scale, out=out)

        row = {"batch": B, "ctx": ctx, "kv_MB": round(kv_mb, 1)}
        for name, fn, mode in (("fused", fused, None), ("rope", rope, None),
                               ("plain", attn, 0), ("pipe", attn, 1)):
            old = ops.decode_pipelined(mode) if mode is not None else None
            # R calls per graph: one replay's launch latency (~10-20 us of host time that the
            # events around a replay also measure) is spread over R kernels
            def rep(fn=fn):
                for _ in range(R):
                    fn()
            try:
                ms = ops.benchmark(rep, iters=a.reps, warmup=1, graph=True) / R
            finally:
                if old is not None:
                    ops.decode_pipelined(old)
            us = ms * 1e3
            row[name + "_us"] = round(us, 2)
            if name != "rope":
                row[name + "_TBps"] = round(kv_mb / us, 3)          # MB / us = TB/s
        print(json.dumps(row), flush=True)
        del kc, vc


if __name__ == "__main__":
    main()
