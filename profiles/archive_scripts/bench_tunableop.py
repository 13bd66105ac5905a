#!/usr/bin/env python3
"""Prefill-sized GEMMs (Llama-3-8B, 512 prompts x 32 tokens) on hipBLASLt: default heuristic
vs PyTorch TunableOp (which times every hipBLASLt/rocBLAS solution for the shape once).
Prints one JSON line per shape: default_us, tuned_us."""
import json
import sys
import time

import torch

SHAPES = [(16384, 6144, 4096), (16384, 4096, 4096), (16384, 28672, 4096), (16384, 4096, 14336)]


def bench(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters * 1e6


def main():
    out_csv = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/tunableop_results.csv"
    dev = torch.device("cuda")
    res = {}
    data = {}
    for (M, N, K) in SHAPES:
        x = (torch.randn(M, K, device=dev) * 0.5).to(torch.bfloat16)
        w = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
        data[(M, N, K)] = (x, w)
        res[(M, N, K)] = {"default_us": bench(lambda: torch.matmul(x, w.t()))}
    tun = torch.cuda.tunable
    tun.enable(True)
    tun.tuning_enable(True)
    tun.set_filename(out_csv)
    tun.set_max_tuning_duration(2000)      # ms per shape
    for (M, N, K), (x, w) in data.items():
        t0 = time.perf_counter()
        torch.matmul(x, w.t())
        torch.cuda.synchronize()
        res[(M, N, K)]["tune_s"] = time.perf_counter() - t0
    tun.tuning_enable(False)
    for (M, N, K), (x, w) in data.items():
        res[(M, N, K)]["tuned_us"] = bench(lambda: torch.matmul(x, w.t()))
    pass                                  # results file written by TunableOp itself
    for k, v in res.items():
        fl = 2 * k[0] * k[1] * k[2]
        v["default_tflops"] = fl / v["default_us"] / 1e6
        v["tuned_tflops"] = fl / v["tuned_us"] / 1e6
        print(json.dumps({"M": k[0], "N": k[1], "K": k[2], **{a: round(b, 2) for a, b in v.items()}}),
              flush=True)


if __name__ == "__main__":
    main()
