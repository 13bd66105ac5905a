#!/usr/bin/env python3
"""Where a K-tile of the two-barrier 4-wave GEMM spends its cycles: runs the diagnostic
tile 48 (tile 45 + s_memtime stamps, gemm.hip STAMP) on prefill shapes and prints each
segment's share of the stamped K loop (per workgroup sums, averaged). Read the shares, not
the total: every stamp drains the LDS reads the real kernel keeps in flight."""
import argparse
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

SEGS = ["mfma0-19+F1reads", "B1", "dma_window(80 mfma)", "mfma100-103", "B2",
        "mfma104-127+F0reads"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/stamp_gemm4w.jsonl")
    a = ap.parse_args()
    from distributed_llm_inferencing_amd import ops
    from distributed_llm_inferencing_amd.ops import gemm as G
    dev = torch.device("cuda")
    torch.manual_seed(0)
    recs = []
    for M, N, K in ((8192, 8192, 8192), (16384, 6144, 4096), (16384, 4096, 14336)):
        x = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
        w = (torch.rand(N, K, device=dev) * 2 - 1).mul_(0.05).to(torch.bfloat16)
        tiles = (M // 256) * (N // 256)
        ws = torch.zeros(tiles * 8, dtype=torch.int64, device=dev)
        out = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
        ref = ops._gemm_native(x, w, "none", plan=G.GemmPlan("dli", 45, 1))
        for _ in range(3):
            ops._native_call("dli_gemm", ops._p(x), x.stride(0), ops._p(w), w.stride(0),
                             ops._p(out), out.stride(0), M, N, K, G.EPI["none"], 48, 1, ops._p(None),
                             ops._p(ws), ops._p(None), 1, ops._st())
        torch.cuda.synchronize()
        same = bool(torch.equal(out, ref))
        v = ws.view(tiles, 8).double()
        seg = v[:, :6].mean(0)
        tot = float(seg.sum())
        nk = int(v[0, 6].item())
        rec = {"M": M, "N": N, "K": K, "k_tiles": nk, "same_as_tile45": same,
               "cycles_per_ktile": round(tot / max(nk, 1), 1),
               "share": {SEGS[i]: round(float(seg[i]) / tot, 4) for i in range(6)},
               "cycles_per_ktile_by_segment": {SEGS[i]: round(float(seg[i]) / max(nk, 1), 1)
                                               for i in range(6)}}
        print(json.dumps(rec), flush=True)
        recs.append(rec)
    Path(a.out).parent.mkdir(parents=True, exist_ok=True)
    with open(a.out, "w") as f:
        for r in recs:
            f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
