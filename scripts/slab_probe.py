#!/usr/bin/env python3
"""Split-K slab-store probe at the M = 512 decode shapes: time each projection GEMM (slabs
only, as the fused consumers call it) with fp32 partials (mode 0), bf16 partials (mode 4)
and no partial store at all (mode 5, timing only), cold weights, graph replays; plus the
add + RMSNorm reduce reading 8 / 4 / 2 fp32 slabs. Prints JSON lines."""
import json
import sys

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(
    __import__("os").path.abspath(__file__))))
from distributed_llm_inferencing_amd import ops                     # noqa: E402
from distributed_llm_inferencing_amd.ops import _native as N, gemm as G  # noqa: E402

dev = torch.device("cuda", 0)
lib = N.require_native()
lib.dli_gemm_set_slab_store.argtypes = [__import__("ctypes").c_int]
M = 512
shapes = [("down", 4096, 14336, 22, 8), ("down", 4096, 14336, 28, 4),
          ("o", 4096, 4096, 28, 4), ("o", 4096, 4096, 22, 8),
          ("qkv", 6144, 4096, 23, 2), ("qkv", 6144, 4096, 25, 4)]
x = (torch.randn(M, 14336, device=dev) * 0.5).to(torch.bfloat16)
for name, Nn, K, tile, sp in shapes:
    w0 = (torch.randn(Nn, K, device=dev) * 0.02).to(torch.bfloat16)
    nc = max(2, min(16, -(-(1 << 30) // (w0.numel() * 2))))
    ws_ = [w0] + [w0.clone() for _ in range(nc - 1)]
    xa = x[:, :K].contiguous()
    slab = G.workspace(dev, sp * M * Nn * 4)
    for mode in (0, 4, 5, 0):
        lib.dli_gemm_set_slab_store(mode)

        def run():
            for w in ws_:
                N.call("dli_gemm", xa.data_ptr(), xa.stride(0), w.data_ptr(), w.stride(0), None,
                       Nn, M, Nn, K, 0, tile, sp, None, slab.data_ptr(), None, 1, N.stream_ptr())
        us = ops.benchmark(run, iters=10, warmup=2, graph=True) * 1e3 / len(ws_)
        print(json.dumps({"gemm": name, "N": Nn, "K": K, "tile": tile, "splits": sp,
                          "slab_mode": mode, "us": round(us, 2)}), flush=True)
    lib.dli_gemm_set_slab_store(0)
    del ws_
# the reduce alone (fp32 slabs; 4 fp32 slabs = the bytes of 8 bf16 ones)
res = torch.zeros(M, 4096, dtype=torch.bfloat16, device=dev)
nw = torch.ones(4096, dtype=torch.bfloat16, device=dev)
out = torch.empty_like(res)
for sp in (8, 4, 2):
    slab = G.workspace(dev, 8 * M * 4096 * 4)
    def red():
        N.call("dli_splitk_add_rmsnorm", out.data_ptr(), res.data_ptr(), slab.data_ptr(), sp, M,
               4096, nw.data_ptr(), 1e-5, 0, N.stream_ptr())
    us = ops.benchmark(red, iters=20, warmup=3, graph=True) * 1e3
    print(json.dumps({"reduce": "add_rmsnorm", "splits_fp32": sp, "us": round(us, 2)}),
          flush=True)
