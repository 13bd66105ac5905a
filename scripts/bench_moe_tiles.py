#!/usr/bin/env python3
"""Every grouped-GEMM candidate plan for the Mixtral 8x7B MoE projections at one decode
batch, timed as ``ops.gemm.autotune_grouped`` times them (seeded multinomial routing of
``rows = batch * top_k`` permuted rows over the experts; the expert weights together exceed
the Infinity Cache, so each call streams them from HBM). Prints one JSON line per plan,
sorted by time, with the achieved weight-streaming bandwidth.

    python scripts/bench_moe_tiles.py [--batch 512] [--which down,gate_up]
    python scripts/bench_moe_tiles.py --batch 16384 --tiles 22,45   # prefill-sized experts

With ``--tiles`` only those tiles run, and the grid is bounded by the largest expert's rows
(the eager prefill path of ``ops.moe_mlp``) instead of all rows.
"""
import argparse
import itertools
import json
import sys
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--which", default="down,gate_up")
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--tiles", default="")
    a = ap.parse_args()
    only = [int(t) for t in a.tiles.split(",") if t]
    from distributed_llm_inferencing_amd import ops
    from distributed_llm_inferencing_amd.ops import gemm as G
    dev = torch.device("cuda")
    E, D, F = 8, 4096, 14336
    rows = a.batch * 2
    counts = np.random.default_rng(1234).multinomial(rows, [1.0 / E] * E).tolist()
    off = torch.tensor([0] + list(itertools.accumulate(counts)), dtype=torch.int32, device=dev)
    for which in a.which.split(","):
        N, K, epi = (D, F, "none") if which == "down" else (2 * F, D, "silu_mul")
        w = (torch.randn(E, N, K, device=dev) * 0.02).to(torch.bfloat16)
        x = (torch.randn(rows, K, device=dev) * 0.5).to(torch.bfloat16)
        out = []
        rpg = max(counts) if only else rows
        ones = torch.ones(rows, 1, dtype=torch.float32, device=dev)
        ident = torch.arange(rows, dtype=torch.int32, device=dev).view(-1, 1)
        comb = torch.empty(rows, N, dtype=torch.bfloat16, device=dev)
        for tile in (only or sorted(G.TILES)):
            if not only and (G.TILES[tile][0] > 2 * max(64, rows // E + 32)
                             or not G.tile_ok(tile, epi)):
                continue
            for splits in (1, 2, 4):
                if splits > 1 and not (K % (64 * splits) == 0 and K // splits >= 2048):
                    continue
                p = G.GemmPlan("dli", tile, splits)
                # split down plans on the fp16-slab tiles: the fused slab combine as the
                # model runs it (ops.moe_down_combine; one pick per row, weight 1)
                fused = which == "down" and ops.moe_slab_plan(p) and not only

                def run(p=p, fused=fused):
                    if fused:
                        ops.moe_down_combine(x, w, off, rows, p, ones, ident, comb)
                    else:
                        ops._gemm_native(x, w, epi, plan=p, groups=E, group_off=off,
                                         rows_per_group=rpg)
                try:
                    ms = ops.benchmark(run, iters=a.iters, warmup=1)
                except Exception as e:  # noqa: BLE001
                    out.append({"which": which, "tile": tile, "splits": splits,
                                "error": str(e)[:60]})
                    continue
                out.append({"which": which, "rows": rows, "tile": tile,
                            "bm_bn": G.TILES.get(tile), "splits": splits, "fused": fused,
                            "us": round(ms * 1e3, 1),
                            "tflops": round(2.0 * rows * N * K / (ms * 1e-3) / 1e12, 1),
                            "weight_TBps": round(w.numel() * 2 / (ms * 1e-3) / 1e12, 2)})
        for r in sorted(out, key=lambda r: r.get("us", 1e9)):
            print(json.dumps(r), flush=True)
        del w


if __name__ == "__main__":
    main()
