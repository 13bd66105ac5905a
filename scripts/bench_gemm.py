#!/usr/bin/env python3
"""GEMM microbenchmark on the Llama-3 projection shapes: every dli MFMA plan vs hipBLASLt
(torch.matmul). Random bf16 operands (cdna_hip_programming.md §5.4 rule 25). Writes JSON."""
import argparse
import json
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from distributed_llm_inferencing_amd import ops  # noqa: E402
from distributed_llm_inferencing_amd.ops import gemm as G  # noqa: E402

SHAPES = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096),
          "down": (4096, 14336), "lm_head": (128256, 4096)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ms", default="1,16,64,128,256,512,2048,8192")
    ap.add_argument("--out", default="gpurun_out/gemm_bench.json")
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda")
    res = []
    for name, (N, K) in SHAPES.items():
        w = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
        for M in [int(x) for x in a.ms.split(",")]:
            if name == "lm_head" and M > 512:
                continue
            x = torch.randn(M, K, device=dev).to(torch.bfloat16)
            epis = ["none", "silu_mul"] if name == "gate_up" else ["none"]
            for epi in epis:
                rows = []
                for p in G.candidate_plans(M, N, K, epi):
                    if p.backend == "hipblaslt":
                        fn = lambda: torch.matmul(x, w.t())  # noqa: E731
                    else:
                        fn = lambda p=p: ops._gemm_native(x, w, epi, plan=p)  # noqa: E731
                    ms = ops.benchmark(fn, iters=a.iters, warmup=3)
                    rows.append((ms, p))
                rows.sort(key=lambda r: r[0])
                best = rows[0]
                blas = [r for r in rows if r[1].backend == "hipblaslt"]
                dli = [r for r in rows if r[1].backend == "dli"]
                heur = G._heuristic(M, N, K, epi)
                heur_ms = next((r[0] for r in rows if r[1] == heur), None)
                flops = 2 * M * N * K
                byts = 2 * (N * K + M * K + M * N)
                rec = {"name": name, "M": M, "N": N, "K": K, "epi": epi,
                       "best": {"backend": best[1].backend, "tile": best[1].tile,
                                "splits": best[1].splits, "ms": best[0]},
                       "best_dli_ms": dli[0][0] if dli else None,
                       "best_dli": [dli[0][1].tile, dli[0][1].splits] if dli else None,
                       "heuristic_ms": heur_ms,
                       "hipblaslt_ms": blas[0][0] if blas else None,
                       "dli_tflops": flops / dli[0][0] / 1e9 if dli else None,
                       "dli_tbps": byts / dli[0][0] / 1e9 if dli else None}
                res.append(rec)
                print(json.dumps(rec), flush=True)
    Path(a.out).parent.mkdir(parents=True, exist_ok=True)
    Path(a.out).write_text(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
