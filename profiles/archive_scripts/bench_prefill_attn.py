#!/usr/bin/env python3
"""Causal GQA prefill attention (Llama-3 32/8 heads, hd 128) at long prompt lengths: the
256-row 32x32x16 kernel vs the 64-row 16x16x32 kernel on the same inputs, interleaved rounds
in one process; causal TFLOP/s = 2 * 2 * L^2/2 * hd * Hq / t. Checks both against each other
and a slice against the fp32 reference."""
import argparse
import json
import math
import statistics
import sys
from pathlib import Path

import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from distributed_llm_inferencing_amd import ops  # noqa: E402
from distributed_llm_inferencing_amd.ops import reference as R  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lens", default="512,2048,8064")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--out", default="gpurun_out/prefill_attn.json")
    a = ap.parse_args()
    dev = torch.device("cuda")
    hq, hkv, hd = 32, 8, 128
    sc = 1 / math.sqrt(hd)
    torch.manual_seed(0)
    res = []
    for L in [int(x) for x in a.lens.split(",")]:
        qkv = torch.randn(L, (hq + 2 * hkv) * hd, device=dev).to(torch.bfloat16)
        cu = torch.tensor([0, L], dtype=torch.int32, device=dev)
        run = {}
        for name, thr in (("long32", 1), ("short16", 1 << 30)):
            def fn(thr=thr):
                old = ops.prefill_long_min_len(thr)
                o = ops.prefill_attention(qkv, cu, L, hq, hkv, hd, sc)
                ops.prefill_long_min_len(old)
                return o
            run[name] = fn
        outs = {k: f() for k, f in run.items()}
        torch.cuda.synchronize()
        diff = (outs["long32"].float() - outs["short16"].float()).abs().max().item()
        # fp32 reference on 2 heads (memory)
        q, k, v = R.split_qkv(qkv, hq, hkv, hd)
        ref = R.prefill_attention(q[:, :2].contiguous(), k[:, :1].contiguous(),
                                  v[:, :1].contiguous(), cu, sc).reshape(L, -1)
        err = (outs["long32"][:, : 2 * hd].float() - ref.float()).abs().max().item()
        times = {k: [] for k in run}
        for _ in range(a.rounds):
            for k, f in run.items():
                times[k].append(ops.benchmark(f, iters=5, warmup=1) * 1e3)
        flops = 2.0 * L * L * hd * hq       # causal: 2 products x L^2/2 x 2 flop
        rec = {"L": L, "max_diff_long_vs_short": diff, "max_err_long_vs_fp32": err}
        for k, v_ in times.items():
            rec[f"us_{k}"] = statistics.median(v_)
            rec[f"tflops_{k}"] = flops / (statistics.median(v_) * 1e-6) / 1e12
        res.append(rec)
        print(json.dumps(rec), flush=True)
    Path(a.out).parent.mkdir(parents=True, exist_ok=True)
    Path(a.out).write_text(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
