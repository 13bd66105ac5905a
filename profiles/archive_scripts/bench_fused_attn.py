"""Same-box A/B of the fused decode attention (dli_decode_attention_fused: split-K QKV slab
sum + RoPE + KV write + paged attention) between builds: the in-tree library and any
--lib ab/lib*.so built from another revision by scripts/ab_lib.sh. Llama-3-8B shapes
(32 / 8 heads, hd 128, block 16), every sequence at the same context, random block tables.
Builds are timed interleaved (A B A B ...) and their outputs compared bit for bit.
Prints one JSON line per (build, ctx, B)."""
from __future__ import annotations

import argparse
import ctypes
import json
import math
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from distributed_llm_inferencing_amd.ops import reference as R  # noqa: E402

P, I, F = ctypes.c_void_p, ctypes.c_int, ctypes.c_float
SIG = [P, P, I, P, P, P, P, P, P, I, P, I, I, I, I, I, F, P]


def load(path):
    lib = ctypes.CDLL(path)
    fn = lib.dli_decode_attention_fused
    fn.argtypes, fn.restype = SIG, I
    return fn


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", action="append", default=[])
    ap.add_argument("--B", default="512")
    ap.add_argument("--ctx", default="33,66,100")
    ap.add_argument("--splits", type=int, default=2)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    from distributed_llm_inferencing_amd.ops import _native as N
    libs = {"tree": N.LIB_PATH} | {os.path.basename(p): p for p in a.lib}
    fns = {k: load(str(v)) for k, v in libs.items()}
    dev = torch.device("cuda")
    hq, hkv, hd, bs = 32, 8, 128, 16
    Nn = (hq + 2 * hkv) * hd
    scale = 1 / math.sqrt(hd)
    cs = R.rope_cos_sin(4096, hd, 500000.0, device=dev)
    st = torch.cuda.current_stream().cuda_stream
    g = torch.Generator(device=dev).manual_seed(0)
    for B in [int(x) for x in a.B.split(",")]:
        for ctx in [int(c) for c in a.ctx.split(",")]:
            nb = -(-ctx // bs)
            nblk = B * nb + 8
            kc = (torch.randn(nblk, hkv, bs, hd, device=dev, generator=g) * 0.5).to(torch.bfloat16)
            vc = (torch.randn(nblk, hkv, bs, hd, device=dev, generator=g) * 0.5).to(torch.bfloat16)
            tables = torch.randperm(nblk, device=dev, generator=g)[:B * nb].to(torch.int32)
            tables = tables.view(B, nb).contiguous()
            ctxs = torch.full((B,), ctx, dtype=torch.int32, device=dev)
            pos = (ctxs - 1).contiguous()
            slots = (tables[:, (ctx - 1) // bs] * bs + (ctx - 1) % bs).to(torch.int32).contiguous()
            ws = torch.randn(max(a.splits, 1), B, Nn, device=dev, generator=g) * 0.1
            src = ws if a.splits > 0 else ws[0].to(torch.bfloat16)
            outs, times = {}, {k: [] for k in fns}
            for _ in range(a.rounds):
                for name, fn in fns.items():
                    out = torch.empty(B, hq * hd, dtype=torch.bfloat16, device=dev)

                    def call():
                        rc = fn(out.data_ptr(), src.data_ptr(), a.splits, pos.data_ptr(),
                                slots.data_ptr(), cs.data_ptr(), kc.data_ptr(), vc.data_ptr(),
                                tables.data_ptr(), tables.stride(0), ctxs.data_ptr(), B, hq,
                                hkv, hd, bs, scale, st)
                        assert rc == 0, rc
                    for _ in range(5):
                        call()
                    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    s.record()
                    for _ in range(a.iters):
                        call()
                    e.record()
                    torch.cuda.synchronize()
                    times[name].append(s.elapsed_time(e) * 1e3 / a.iters)
                    outs[name] = out
            ref = outs["tree"]
            kv = 2 * B * hkv * ctx * hd * 2
            for name in fns:
                us = min(times[name])
                print(json.dumps({"build": name, "B": B, "ctx": ctx, "splits": a.splits,
                                  "us": round(us, 2), "all_us": [round(t, 2) for t in times[name]],
                                  "kv_tbs": round(kv / us / 1e6, 2),
                                  "equal_to_tree": bool(torch.equal(outs[name], ref))}),
                      flush=True)


if __name__ == "__main__":
    main()
