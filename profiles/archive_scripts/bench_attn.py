#!/usr/bin/env python3
"""Decode attention at the bench's shapes (Llama-3-8B GQA 32/8, hd 128, block 16, B = 512,
every sequence at the same context, as in a bench wave): time + HBM rate + max error vs the
fp32 PyTorch reference of the same op."""
import argparse
import json
import math
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from distributed_llm_inferencing_amd import ops  # noqa: E402
from distributed_llm_inferencing_amd.ops import reference as R  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=512)
    ap.add_argument("--ctx", default="33,66,100,1000")
    ap.add_argument("--out", default="gpurun_out/attn.json")
    a = ap.parse_args()
    dev = torch.device("cuda")
    hq, hkv, hd, bs = 32, 8, 128, 16
    torch.manual_seed(0)
    res = []
    for ctx in [int(c) for c in a.ctx.split(",")]:
        B = a.B if ctx <= 128 else 64
        nb = -(-ctx // bs)
        nblk = B * nb + 8
        kc = (torch.randn(nblk, hkv, bs, hd, device=dev) * 0.5).to(torch.bfloat16)
        vc = (torch.randn(nblk, hkv, bs, hd, device=dev) * 0.5).to(torch.bfloat16)
        perm = torch.randperm(nblk, device=dev)[: B * nb].view(B, nb).to(torch.int32)
        W = max(nb, 8)
        tables = torch.zeros(B, W, dtype=torch.int32, device=dev)
        tables[:, :nb] = perm
        lens = torch.full((B,), ctx, dtype=torch.int32, device=dev)
        qkv = torch.randn(B, (hq + 2 * hkv) * hd, device=dev).to(torch.bfloat16)
        sc = 1 / math.sqrt(hd)
        ref = R.decode_attention(qkv[:, : hq * hd].reshape(B, hq, hd).float(), kc.float(),
                                 vc.float(), tables, lens, sc).reshape(B, hq * hd)
        kv_bytes = B * ctx * hkv * hd * 2 * 2
        rec = {"B": B, "ctx": ctx}
        times = {0: [], 1: []}
        for v in (0, 1):                   # one-tile-per-round vs pipelined kernel
            ops.decode_pipelined(v)
            out = ops.decode_attention(qkv, kc, vc, tables, lens, ctx, hq, hkv, hd, sc)
            rec[f"max_err_{v}"] = (out.float() - ref.float()).abs().max().item()
        for _ in range(5):                 # interleaved rounds
            for v in (0, 1):
                ops.decode_pipelined(v)
                times[v].append(ops.benchmark(lambda: ops.decode_attention(
                    qkv, kc, vc, tables, lens, ctx, hq, hkv, hd, sc), iters=20))
        ops.decode_pipelined(-1)
        for v, name in ((0, "round"), (1, "pipe")):
            ms = sorted(times[v])[len(times[v]) // 2]
            rec[f"us_{name}"] = ms * 1e3
            rec[f"TBps_{name}"] = kv_bytes / ms / 1e9
        res.append(rec)
        print(json.dumps(rec), flush=True)
    Path(a.out).parent.mkdir(parents=True, exist_ok=True)
    Path(a.out).write_text(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
