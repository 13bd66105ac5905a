#!/usr/bin/env python3
"""Decode attention at the bench's shapes (mixed context 33..100) for forced KV split counts:
does splitting the context across more waves help when B*Hkv already fills the chip?"""
import json
import math
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from distributed_llm_inferencing_amd import ops  # noqa: E402


def main():
    dev = torch.device("cuda")
    hq, hkv, hd, bs, W = 32, 8, 128, 16, 8
    torch.manual_seed(0)
    for B in (512, 256, 64):
        lens_l = torch.randint(33, 100, (B,)).tolist()
        nblk = sum(-(-n // bs) for n in lens_l) + 8
        kc = (torch.randn(nblk, hkv, bs, hd, device=dev) * 0.5).to(torch.bfloat16)
        vc = (torch.randn(nblk, hkv, bs, hd, device=dev) * 0.5).to(torch.bfloat16)
        perm = torch.randperm(nblk).tolist()
        tables, o = [], 0
        for n in lens_l:
            nb = -(-n // bs)
            tables.append(perm[o:o + nb] + [0] * (W - nb))
            o += nb
        tables = torch.tensor(tables, device=dev, dtype=torch.int32)
        lens = torch.tensor(lens_l, device=dev, dtype=torch.int32)
        qkv = torch.randn(B, (hq + 2 * hkv) * hd, device=dev).to(torch.bfloat16)
        sc = 1 / math.sqrt(hd)
        ref = ops.decode_attention(qkv, kc, vc, tables, lens, W * bs, hq, hkv, hd, sc,
                                   num_splits=1).float()
        for ns in (1, 2, 4):
            out = ops.decode_attention(qkv, kc, vc, tables, lens, W * bs, hq, hkv, hd, sc,
                                       num_splits=ns)
            err = (out.float() - ref).abs().max().item()
            ms = ops.benchmark(lambda: ops.decode_attention(qkv, kc, vc, tables, lens, W * bs,
                                                            hq, hkv, hd, sc, num_splits=ns),
                               iters=50)
            print(json.dumps({"B": B, "splits": ns, "us": round(ms * 1e3, 2),
                              "default_splits": ops.decode_num_splits(B, hkv, W * bs),
                              "max_diff_vs_1": err}), flush=True)


if __name__ == "__main__":
    main()
