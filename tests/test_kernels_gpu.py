"""T3 kernel golden tests: every HIP kernel vs the PyTorch fp32 reference of the same op
(ops/reference.py), on the GPU. Run on an MI355X via gpurun."""
import math
import os

import numpy as np
import pytest
import torch

from distributed_llm_inferencing_amd import ops
from distributed_llm_inferencing_amd.ops import gemm as G
from distributed_llm_inferencing_amd.ops import reference as R

pytestmark = pytest.mark.gpu
BF = torch.bfloat16


def rnd(*shape, dev, scale=1.0, dtype=BF):
    return (torch.randn(*shape, device=dev) * scale).to(dtype)


def close(a, b, rtol=2e-2, atol=2e-2):
    a, b = a.float(), b.float()
    err = (a - b).abs().max().item()
    tol = atol + rtol * b.abs().max().item()
    assert err <= tol, f"max err {err} > tol {tol}"


@pytest.mark.parametrize("T,D", [(1, 256), (7, 768), (64, 4096), (33, 8192)])
def test_rmsnorm_and_fused_add(gpu, T, D):
    torch.manual_seed(0)
    x, r, w = rnd(T, D, dev=gpu), rnd(T, D, dev=gpu), rnd(D, dev=gpu)
    close(ops.rmsnorm(x, w, 1e-5), R.rmsnorm(x, w, 1e-5))
    res = r.clone()
    out = ops.add_rmsnorm(x, res, w, 1e-5)
    ref_out, ref_res = R.fused_add_rmsnorm(x, r, w, 1e-5)
    close(out, ref_out)
    assert torch.equal(res, ref_res)
    copy = torch.empty_like(x)
    ops.rmsnorm(x, w, 1e-5, residual_copy=copy)
    assert torch.equal(copy, x)


@pytest.mark.parametrize("T,D", [(5, 768), (40, 256)])
def test_layernorm_and_fused_add(gpu, T, D):
    torch.manual_seed(1)
    x, r, w, b = rnd(T, D, dev=gpu), rnd(T, D, dev=gpu), rnd(D, dev=gpu), rnd(D, dev=gpu)
    close(ops.layernorm(x, w, b, 1e-5), R.layernorm(x, w, b, 1e-5))
    res = r.clone()
    out = ops.add_layernorm(x, res, w, b, 1e-5)
    ro, rr = R.fused_add_layernorm(x, r, w, b, 1e-5)
    close(out, ro)
    assert torch.equal(res, rr)


def test_embedding(gpu):
    tab, pos = rnd(1000, 256, dev=gpu), rnd(64, 256, dev=gpu)
    ids = torch.randint(0, 1000, (37,), device=gpu, dtype=torch.int32)
    p = torch.randint(0, 64, (37,), device=gpu, dtype=torch.int32)
    assert torch.equal(ops.embedding(ids, tab), R.embedding(ids, tab))
    close(ops.embedding(ids, tab, pos, p), R.embedding(ids, tab, pos, p), rtol=1e-2, atol=1e-2)


GEMM_SHAPES = [(1, 256, 256), (7, 768, 2304), (64, 4096, 4096), (100, 1000, 512),
               (256, 6144, 4096), (300, 4096, 14336), (1024, 512, 1024), (33, 50257, 768)]


@pytest.mark.parametrize("M,N,K", GEMM_SHAPES)
def test_gemm_bf16_all_tiles(gpu, M, N, K):
    torch.manual_seed(2)
    x, w = rnd(M, K, dev=gpu), rnd(N, K, dev=gpu, scale=0.05)
    ref = R.linear(x, w, out_dtype=torch.float32)
    for tile in G.TILES:
        # split 8: (split, tile) grids whose size is not a multiple of the 8 XCDs exercise
        # the split-major block remap (gemm.hip split_tile)
        for splits in (1, 2, 4, 8):
            if K % (64 * splits):
                continue
            if tile == 55 and (splits > 1 or K % 128):      # persistent: unsplit, even K-tiles
                continue
            out = ops._gemm_native(x, w, "none", plan=G.GemmPlan("dli", tile, splits))
            close(out, ref, rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("tile", [26, 28])
@pytest.mark.parametrize("M,N,K,epi", [(512, 28672, 4096, "silu_mul"), (500, 2240, 14336, "none"),
                                       (1000, 7168, 1024, "f32"), (512, 4096, 14336, "none")])
def test_gemm_256x224_pingpong(gpu, M, N, K, epi, tile):
    """Tiles 26 (256x224 ping-pong) and 28 (256x128 ping-pong) at the Llama-3 gate/up and
    down decode shapes and with long K / partial M tiles, against the fp32 reference."""
    torch.manual_seed(5)
    x, w = rnd(M, K, dev=gpu), rnd(N, K, dev=gpu, scale=0.05)
    if epi == "silu_mul":
        ref = R.silu_mul(R.linear(x, w).float().to(BF))
    else:
        ref = R.linear(x, w, out_dtype=torch.float32)
    for splits in (1, 2, 4):
        if K % (64 * splits):
            continue
        out = ops._gemm_native(x, w, epi, plan=G.GemmPlan("dli", tile, splits))
        close(out, ref, rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("M,N,K,epi", [(2048, 6144, 4096, "none"), (4096, 4096, 4096, "none"),
                                       (8192, 28672, 4096, "silu_mul"),
                                       (16384, 4096, 14336, "none"), (512, 28672, 4096, "silu_mul"),
                                       (1100, 4096, 14336, "none"), (777, 50257, 4096, "f32"),
                                       (300, 2304, 768, "bias_gelu")])
def test_gemm_4wave_persistent(gpu, M, N, K, epi):
    """Tile 55: the two-barrier 4-wave kernel as a persistent grid (one workgroup per CU walks
    tiles; the next tile's first K-tiles are staged in the current tile's last two). Shapes
    with one tile per workgroup (M = 2048 QKV: 192 tiles), many (gate/up at 8192: 3,584
    tiles, 14 per workgroup), partial row / column tiles and every epilogue, against the fp32
    reference; bitwise equal to tile 45 (same K order per output); odd K-tile counts and
    split-K are refused."""
    torch.manual_seed(11)
    x, w = rnd(M, K, dev=gpu), rnd(N, K, dev=gpu, scale=0.05)
    bias = rnd(N, dev=gpu) if epi == "bias_gelu" else None
    if epi == "silu_mul":
        ref = R.silu_mul(R.linear(x, w).float().to(BF))
    elif epi == "bias_gelu":
        ref = R.gelu_tanh(R.linear(x, w).float() + bias.float())
    else:
        ref = R.linear(x, w, out_dtype=torch.float32)
    t45 = ops._gemm_native(x, w, epi, plan=G.GemmPlan("dli", 45, 1), bias=bias)
    for rep in range(3):
        out = ops._gemm_native(x, w, epi, plan=G.GemmPlan("dli", 55, 1), bias=bias)
        err = (out.float() - ref.float()).abs()
        bad = err > 2e-2 + 2e-2 * ref.float().abs().max()
        assert not bool(bad.any()), (
            f"rep {rep}: {int(bad.sum())} bad elements, rows "
            f"{torch.unique(torch.nonzero(bad)[:, 0])[:16].tolist()}, cols "
            f"{torch.unique(torch.nonzero(bad)[:, 1])[:16].tolist()}, max {float(err.max())}")
        assert torch.equal(out, t45)
    with pytest.raises(Exception):
        ops._gemm_native(x, w, epi, plan=G.GemmPlan("dli", 55, 2), bias=bias)
    if K % 128 == 0:
        x2, w2 = x[:, :K - 64].contiguous(), w[:, :K - 64].contiguous()   # odd K-tile count
        with pytest.raises(Exception):
            ops._gemm_native(x2, w2, epi, plan=G.GemmPlan("dli", 55, 1), bias=bias)


@pytest.mark.parametrize("tile", [int(t) for t in os.environ.get("DLI_TEST_4W_TILES",
                                                                  "34,41,45").split(",")])
@pytest.mark.parametrize("M,N,K,epi", [(2048, 6144, 4096, "none"), (4096, 4096, 4096, "none"),
                                       (8192, 28672, 4096, "silu_mul"),
                                       (16384, 4096, 14336, "none"), (512, 28672, 4096, "silu_mul"),
                                       (1100, 4096, 14336, "none"), (777, 50257, 4096, "f32"),
                                       (300, 2304, 768, "bias_gelu")])
def test_gemm_4wave_256(gpu, M, N, K, epi, tile):
    """The one-wave-per-SIMD 256x256 kernel (tiles 34-37: AGPR-pinned accumulators, buffer
    LDS-DMA with range-checked rows) at the prefill token buckets of the Llama-3-8B
    projections (QKV / O / gate-up / down), a decode batch, partial row and column tiles
    (M = 1100 / 777 / 300, N = 50257) and every epilogue, split-K 1/2/4, against the fp32
    reference."""
    torch.manual_seed(11)
    x, w = rnd(M, K, dev=gpu), rnd(N, K, dev=gpu, scale=0.05)
    bias = rnd(N, dev=gpu) if epi == "bias_gelu" else None
    if epi == "silu_mul":
        ref = R.silu_mul(R.linear(x, w).float().to(BF))
    elif epi == "bias_gelu":
        ref = R.gelu_tanh(R.linear(x, w).float() + bias.float())
    else:
        ref = R.linear(x, w, out_dtype=torch.float32)
    for splits in (1, 2, 4):
        if K % (64 * splits) or (splits > 1 and M * N > (1 << 27)):
            continue
        for rep in range(3):              # a schedule race shows up as an intermittent tile
            out = ops._gemm_native(x, w, epi, plan=G.GemmPlan("dli", tile, splits), bias=bias)
            err = (out.float() - ref.float()).abs()
            bad = err > 2e-2 + 2e-2 * ref.float().abs().max()
            assert not bool(bad.any()), (
                f"tile {tile} split {splits} rep {rep}: {int(bad.sum())} bad elements, rows "
                f"{torch.unique(torch.nonzero(bad)[:, 0])[:16].tolist()}, cols "
                f"{torch.unique(torch.nonzero(bad)[:, 1])[:16].tolist()}, max {float(err.max())}")


@pytest.mark.parametrize("M", [1, 2, 3, 4])
@pytest.mark.parametrize("N,K,epi", [(6144, 4096, "none"), (4096, 14336, "none"),
                                     (28672, 4096, "silu_mul"), (96, 768, "silu_mul"),
                                     (50257, 768, "f32"),
                                     (2304, 768, "bias")])
def test_gemv_skinny(gpu, M, N, K, epi):
    """The M <= 4 weight-streaming GEMM (tiles 29-33) against the fp32 reference: every
    epilogue, split-K 1/2/4 (reduce kernel), a K (768) that is not a multiple of the
    512-element wave step, and a final partial row block (N = 50257). Tile 29 (M = 1 SiLU*up
    on the 16-row grid, 8 gate + 8 up rows per workgroup) runs on the gate/up shapes."""
    torch.manual_seed(7)
    x, w, b = rnd(M, K, dev=gpu), rnd(N, K, dev=gpu, scale=0.05), rnd(N, dev=gpu)
    if epi == "silu_mul":
        ref = R.silu_mul(R.linear(x, w).float().to(BF))
    elif epi == "f32":
        ref = R.linear(x, w, out_dtype=torch.float32)
    elif epi == "bias":
        ref = R.linear(x, w, b)
    else:
        ref = R.linear(x, w, out_dtype=torch.float32)
    for tile in G.GEMV_TILES:
        if not G.tile_ok(tile, epi) or (tile in G.GEMV_M1_ONLY and M > 1):
            continue
        for splits in (1, 2, 4):
            if K % (64 * splits):
                continue
            out = ops._gemm_native(x, w, epi, bias=b if epi == "bias" else None,
                                   plan=G.GemmPlan("dli", tile, splits))
            close(out, ref, rtol=2e-2, atol=2e-2)
    if epi == "none" and K % 128 == 0:       # split-K slabs into the fused add + RMSNorm
        r0, nw = rnd(M, N, dev=gpu), rnd(N, dev=gpu)
        ref_out, ref_res = R.fused_add_rmsnorm(R.linear(x, w), r0, nw, 1e-5)
        for splits in (2, 4):
            G.set_plan(M, N, K, "splitk", G.GemmPlan("dli", 30, splits))
            res = r0.clone()
            out = ops.linear_add_rmsnorm(x, w, res, nw, 1e-5)
            close(out, ref_out, rtol=2e-2, atol=3e-2)
            close(res, ref_res, rtol=1e-2, atol=2e-2)
        G.clear_plans()


@pytest.mark.parametrize("M", [1, 2, 3, 4])
@pytest.mark.parametrize("N,K", [(4096, 4096), (4096, 14336), (1000, 768)])
def test_gemv_residual_epilogue(gpu, M, N, K):
    """Batch-1 decode O / down projection as one kernel (ops.linear_residual, epi "res"):
    residual += x @ W^T with full K per workgroup == the fp32 reference rounded as
    splitk_add_rmsnorm rounds (GEMM result to bf16, then the add); every tile (30 / 32 / 56 /
    57) gives the same bits, since a row's K order does not depend on the row block; graph
    replays equal eager."""
    torch.manual_seed(5)
    x, w, r0 = rnd(M, K, dev=gpu), rnd(N, K, dev=gpu, scale=0.05), rnd(M, N, dev=gpu)
    ref = (r0.float() + R.linear(x, w, out_dtype=torch.float32).to(BF).float()).to(BF)
    got = None
    plans = G.candidate_plans(M, N, K, "res")
    assert {p.tile for p in plans} >= {30, 56, 57} and all(p.splits == 1 for p in plans)
    for p in plans:
        res = r0.clone()
        ops.linear_residual(x, w, res, plan=p)
        close(res, ref, rtol=1e-2, atol=2e-2)
        if got is None:
            got = res
        assert torch.equal(res, got), p
    res_g = r0.clone()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        ops.linear_residual(x, w, res_g, plan=plans[-1])
    res_g.copy_(r0)
    g.replay()
    torch.cuda.synchronize()
    assert torch.equal(res_g, got)


@pytest.mark.parametrize("M", [1, 2, 4])
@pytest.mark.parametrize("N,K,epi", [(6144, 4096, "splitk"), (28672, 4096, "silu_mul"),
                                     (96, 768, "silu_mul"), (1024, 2048, "none"),
                                     (512, 8192, "none")])
def test_gemv_norm_prologue(gpu, M, N, K, epi):
    """A GEMV whose input is a deferred RMSNorm (ops.NormedRows): its prologue normalises
    the raw residual rows into LDS, then streams the weights. == the fp32 reference of
    (rmsnorm(residual) * w) @ W^T for every prologue tile: bf16 rows, SiLU*up (16-row
    interleaved gate/up weight) and the fp32 split-K slabs the fused QKV consumer reads;
    K = 8192 at M = 4 fills the 64 KB of LDS rows."""
    torch.manual_seed(9)
    r, nw, w = rnd(M, K, dev=gpu), rnd(K, dev=gpu), rnd(N, K, dev=gpu, scale=0.05)
    xn = R.rmsnorm(r, nw, 1e-5)
    h = ops.NormedRows(r, nw, 1e-5)
    ran = 0
    for tile in G.GEMV_PRO_TILES[epi]:
        if tile in G.GEMV_PRO_M1_ONLY and M > 1:
            continue
        if epi == "splitk":
            ref = R.linear(xn, w, out_dtype=torch.float32)
            for splits in (2, 4):
                ws = torch.empty(splits * M * N, dtype=torch.float32, device=gpu)
                assert ops._gemv_prologue(h, w, "splitk", G.GemmPlan("dli", tile, splits), None,
                                          N, ws=ws)
                close(ws.view(splits, M, N).sum(0), ref, rtol=2e-2, atol=2e-2)
                ran += 1
            continue
        ref = (R.silu_mul(R.linear(xn, w).float().to(BF)) if epi == "silu_mul"
               else R.linear(xn, w, out_dtype=torch.float32))
        for splits in (1, 2, 4):             # split K: slabs + the reduce kernel into C
            if K % (64 * splits):
                continue
            G.set_plan(M, N, K, epi, G.GemmPlan("dli", tile, splits))
            try:
                out = ops.linear(h, w, epi=epi)
            finally:
                G.clear_plans()
            close(out, ref, rtol=2e-2, atol=2e-2)
            close(ops.linear_normed(h, w, epi, G.GemmPlan("dli", tile, splits)), ref,
                  rtol=2e-2, atol=2e-2)
            ran += 1
    assert ran
    # a plan without a prologue variant materialises the norm first: same values
    G.set_plan(M, N, K, "none", G.GemmPlan("dli", 2, 1))
    try:
        out = ops.linear(h, w)
    finally:
        G.clear_plans()
    close(out, R.linear(xn, w, out_dtype=torch.float32), rtol=2e-2, atol=2e-2)


def test_prefill_autotune_pins_a_correct_plan(gpu):
    """StageRunner.autotune_prefill's measurement (ops.gemm.autotune over prefill_candidates:
    our 8-phase kernel vs hipBLASLt) pins one plan per shape, and whichever it pins computes
    each consumer (plain, SiLU*up, add + RMSNorm) like the fp32 reference."""
    torch.manual_seed(14)
    G.clear_plans()
    M, K = 2048, 1024
    w_gu, w_o = rnd(2048, K, dev=gpu, scale=0.05), rnd(1024, K, dev=gpu, scale=0.05)
    shapes = [(M, 2048, K, "silu_mul"), (M, 1024, K, "splitk")]
    got = G.autotune(shapes, {(2048, K): w_gu, (1024, K): w_o}, gpu, iters=2, cold_bytes=1,
                     candidates=G.prefill_candidates)
    assert set(got) == set(shapes)
    for (m, n, k, epi), (p, ms) in got.items():
        assert ms > 0 and G.plan(m, n, k, epi) == p
        assert p in G.prefill_candidates(m, n, k, epi)
    x = rnd(M, K, dev=gpu)
    close(ops.linear(x, w_gu, epi="silu_mul"), R.silu_mul(R.linear(x, w_gu).float().to(BF)))
    r0, nw = rnd(M, 1024, dev=gpu), rnd(1024, dev=gpu)
    ref_out, ref_res = R.fused_add_rmsnorm(R.linear(x, w_o), r0, nw, 1e-5)
    res = r0.clone()
    close(ops.linear_add_rmsnorm(x, w_o, res, nw, 1e-5), ref_out, rtol=2e-2, atol=3e-2)
    close(res, ref_res, rtol=1e-2, atol=2e-2)
    G.clear_plans()


def test_gemm_asymmetric_identity(gpu):
    """A = I with asymmetric B catches a transposed C write (cdna_hip_programming.md §3)."""
    n = 128
    eye = torch.eye(n, device=gpu, dtype=BF)
    w = (torch.arange(n * n, device=gpu).reshape(n, n) % 97).to(BF)
    for tile in G.TILES:
        out = ops._gemm_native(eye, w, "none", plan=G.GemmPlan("dli", tile, 1))
        assert torch.equal(out, w.t().contiguous()), tile


@pytest.mark.parametrize("epi", ["none", "f32", "silu_mul", "bias"])
@pytest.mark.parametrize("col0", [3, 4])
def test_gemm_strided_output_views(gpu, epi, col0):
    """The epilogues write four consecutive columns per lane (transposed accumulators) as one
    16-B / 8-B store when C, ldc and N allow it: a column view of a wider buffer at an aligned
    offset (col0 = 4: vector stores with ldc != N) and at a misaligned one (col0 = 3: the
    per-column fallback) must both match the fp32 reference and leave the rest untouched."""
    torch.manual_seed(13)
    M, N, K = 300, 1024, 512
    x, w, b = rnd(M, K, dev=gpu), rnd(N, K, dev=gpu, scale=0.05), rnd(N, dev=gpu)
    if epi == "silu_mul":
        ref = R.silu_mul(R.linear(x, w).float().to(BF))
    elif epi == "bias":
        ref = R.linear(x, w, b)
    else:
        ref = R.linear(x, w, out_dtype=torch.float32)
    out_n = ref.shape[1]
    dt = torch.float32 if epi == "f32" else BF
    for tile in (2, 7, 13, 22, 26, 28):
        if not G.tile_ok(tile, epi):
            continue
        for splits in (1, 2):
            big = torch.full((M, out_n + 8), -7.0, dtype=dt, device=gpu)
            view = big[:, col0:col0 + out_n]
            ops._gemm_native(x, w, epi, bias=b if epi == "bias" else None, out=view,
                             plan=G.GemmPlan("dli", tile, splits))
            close(view, ref, rtol=2e-2, atol=2e-2)
            assert bool((big[:, :col0] == -7.0).all()), (tile, splits)
            assert bool((big[:, col0 + out_n:] == -7.0).all()), (tile, splits)


@pytest.mark.parametrize("epi", ["f32", "silu_mul", "bias_gelu", "bias"])
@pytest.mark.parametrize("M,N,K", [(5, 512, 256), (128, 1024, 512), (260, 3072, 768)])
def test_gemm_epilogues(gpu, epi, M, N, K):
    torch.manual_seed(3)
    x, w, b = rnd(M, K, dev=gpu), rnd(N, K, dev=gpu, scale=0.05), rnd(N, dev=gpu)
    if epi == "silu_mul":
        ref = R.silu_mul(R.linear(x, w).float().to(BF))
    elif epi == "f32":
        ref = R.linear(x, w, out_dtype=torch.float32)
    elif epi == "bias_gelu":
        ref = R.gelu_tanh(R.linear(x, w, b))
    else:
        ref = R.linear(x, w, b)
    for tile in (0, 2, 13, 14, 20, 22, 26):
        for splits in (1, 2):
            out = ops._gemm_native(x, w, epi, bias=b if "bias" in epi else None,
                                   plan=G.GemmPlan("dli", tile, splits))
            close(out, ref, rtol=2e-2, atol=2e-2)
            if epi == "f32":
                assert out.dtype == torch.float32


@pytest.mark.parametrize("tile,splits", [(22, 8), (28, 4), (23, 2), (25, 4), (0, 2)])
@pytest.mark.parametrize("scale", [1.0, 3e4])
def test_fp16_slabs_match_fp32_reference(gpu, monkeypatch, tile, splits, scale):
    """EPI "slab16": the split-K partials of the MFMA families stored as fp16 x 1/16 (half
    the bytes of fp32 slabs) and reduced in fp32 by the fused consumers == the fp32 reference
    within bf16 tolerance, at the M = 512 decode shapes; scale 3e4 puts partial sums at
    1e4-1e5 — beyond fp16's 65504 without the 1/16 scale — and everything stays finite."""
    from distributed_llm_inferencing_amd.ops import reference as RR
    torch.manual_seed(12)
    M, N, K = 512, 4096, 4096
    x, w = rnd(M, K, dev=gpu) * scale, rnd(N, K, dev=gpu, scale=0.02)
    r0, nw = rnd(M, N, dev=gpu) * scale, rnd(N, dev=gpu)
    y = R.linear(x, w)
    ref_out, ref_res = R.fused_add_rmsnorm(y, r0, nw, 1e-5)
    outs = {}
    for s16 in (True, False):
        monkeypatch.setattr(G, "SLAB16", s16)
        G.set_plan(M, N, K, "splitk", G.GemmPlan("dli", tile, splits))
        res = r0.clone()
        out = ops.linear_add_rmsnorm(x, w, res, nw, 1e-5)
        assert torch.isfinite(out).all() and torch.isfinite(res.float()).all()
        close(out, ref_out, rtol=2e-2, atol=3e-2)
        close(res, ref_res, rtol=1e-2, atol=2e-2 * scale)
        outs[s16] = res
    G.clear_plans()
    # fp16 partials differ from fp32 partials by at most a few bf16 ulps of the residual
    d = (outs[True].float() - outs[False].float()).abs()
    assert d.max().item() <= 2 ** -6 * outs[False].float().abs().max().item() + 1e-3
    # the QKV consumer (RoPE + paged KV write) on the same slab format
    hq, hkv, hd = 32, 8, 128
    Nq = (hq + 2 * hkv) * hd
    wq = rnd(Nq, K, dev=gpu, scale=0.02)
    pos = torch.arange(M, device=gpu, dtype=torch.int32) % 100
    slots = torch.arange(M, device=gpu, dtype=torch.int32)
    kc = torch.zeros(M // 16, hkv, 16, hd, dtype=BF, device=gpu)
    vc = torch.zeros_like(kc)
    cs = RR.rope_cos_sin(128, hd, 500000.0, device=gpu)
    if Nq % (splits * 64) == 0 and K % (splits * 64) == 0:
        monkeypatch.setattr(G, "SLAB16", True)
        G.set_plan(M, Nq, K, "splitk", G.GemmPlan("dli", tile, splits))
        qkv = ops.linear_rope_cache(x, wq, pos, slots, cs, kc, vc, hq, hkv, hd)
        G.clear_plans()
        qkv_r = R.linear(x, wq)
        kc_r, vc_r = torch.zeros_like(kc), torch.zeros_like(vc)
        R.rope_and_cache(qkv_r, pos, slots, cs, kc_r, vc_r, hq, hkv, hd)
        close(qkv, qkv_r, rtol=2e-2, atol=3e-2 * scale)
        close(kc, kc_r, rtol=2e-2, atol=3e-2 * scale)
        close(vc, vc_r, rtol=2e-2, atol=3e-2 * scale)


@pytest.mark.parametrize("M,N,K", [(3, 512, 1024), (256, 4096, 4096), (77, 4096, 14336),
                                   (64, 8192, 3072), (5, 2000, 1024), (1, 4096, 4096),
                                   (4, 4096, 14336), (2, 5120, 3072)])
def test_fused_splitk_add_rmsnorm(gpu, M, N, K):
    torch.manual_seed(11)
    x, w = rnd(M, K, dev=gpu), rnd(N, K, dev=gpu, scale=0.02)
    r0, nw = rnd(M, N, dev=gpu), rnd(N, dev=gpu)
    y = R.linear(x, w)                                    # bf16-rounded GEMM output
    ref_out, ref_res = R.fused_add_rmsnorm(y, r0, nw, 1e-5)
    # 2/4/8: compile-time split variants up to N = 4096; 3 and N = 8192 (Llama-3-70B rows,
    # 4 vectors per thread): the runtime-split loop; N = 2000: a partly masked last vector
    for splits in (2, 3, 4, 8) if K % (3 * 64) == 0 else (2, 4, 8):
        G.set_plan(M, N, K, "splitk", G.GemmPlan("dli", 0, splits))
        res = r0.clone()
        out = ops.linear_add_rmsnorm(x, w, res, nw, 1e-5)
        close(out, ref_out, rtol=2e-2, atol=3e-2)
        close(res, ref_res, rtol=1e-2, atol=2e-2)
        res2 = r0.clone()
        assert ops.linear_add_rmsnorm(x, w, res2, None, 1e-5) is None
        assert torch.equal(res2, res)                     # add-only mode: same residual
    G.clear_plans()


@pytest.mark.parametrize("hq,hkv,hd,splits", [(32, 8, 128, 4), (32, 8, 128, 2),
                                              (4, 2, 64, 2), (4, 2, 64, 3)])
def test_fused_splitk_rope_cache(gpu, hq, hkv, hd, splits):
    lens = [5, 17, 1, 40]
    T = sum(lens)
    _, pos, slots, kc, vc, _ = _paged_setup(gpu, lens, hq, hkv, hd, 16)
    K = 1536                                              # divisible into 2, 3 and 4 splits
    N = (hq + 2 * hkv) * hd
    x, w = rnd(T, K, dev=gpu), rnd(N, K, dev=gpu, scale=0.05)
    cs = R.rope_cos_sin(256, hd, 500000.0, device=gpu)
    ref = R.linear(x, w)
    kc1, vc1 = kc.clone(), vc.clone()
    R.rope_and_cache(ref, pos, slots, cs, kc1, vc1, hq, hkv, hd)
    G.set_plan(T, N, K, "splitk", G.GemmPlan("dli", 0, splits))
    out = ops.linear_rope_cache(x, w, pos, slots, cs, kc, vc, hq, hkv, hd)
    G.clear_plans()
    close(out, ref, rtol=2e-2, atol=2e-2)
    close(kc, kc1, rtol=2e-2, atol=2e-2)
    close(vc, vc1, rtol=2e-2, atol=2e-2)


def test_silu_mul_and_bias_act(gpu):
    gu = rnd(9, 2 * 512, dev=gpu)
    close(ops.silu_mul(gu), R.silu_mul(gu))
    x, b = rnd(9, 768, dev=gpu), rnd(768, dev=gpu)
    y = x.clone()
    ops.bias_act_(y, b, "gelu")
    close(y, R.gelu_tanh((x.float() + b.float()).to(BF)))


def _paged_setup(gpu, lens, hq, hkv, hd, bs, nblk=64, seed=4):
    torch.manual_seed(seed)
    T = sum(lens)
    qkv = rnd(T, (hq + 2 * hkv) * hd, dev=gpu)
    pos = torch.cat([torch.arange(n) for n in lens]).to(gpu, torch.int32)
    kc = torch.zeros(nblk, hkv, bs, hd, device=gpu, dtype=BF)
    vc = torch.zeros(nblk, hkv, bs, hd, device=gpu, dtype=BF)
    perm = torch.randperm(nblk).tolist()
    tables, slots, o = [], [], 0
    maxb = max(-(-n // bs) for n in lens)
    for n in lens:
        nb = -(-n // bs)
        blocks = perm[o:o + nb]
        o += nb
        tables.append(blocks + [0] * (maxb - nb))
        slots += [blocks[t // bs] * bs + t % bs for t in range(n)]
    return (qkv, pos, torch.tensor(slots, device=gpu, dtype=torch.int32), kc, vc,
            torch.tensor(tables, device=gpu, dtype=torch.int32))


@pytest.mark.parametrize("hq,hkv,hd", [(32, 8, 128), (12, 12, 64), (4, 2, 64)])
def test_rope_cache(gpu, hq, hkv, hd):
    lens = [5, 17, 1]
    qkv, pos, slots, kc, vc, _ = _paged_setup(gpu, lens, hq, hkv, hd, 16)
    cs = R.rope_cos_sin(256, hd, 500000.0, device=gpu)
    q1, kc1, vc1 = qkv.clone(), kc.clone(), vc.clone()
    R.rope_and_cache(q1, pos, slots, cs, kc1, vc1, hq, hkv, hd)
    q2 = qkv.clone()
    ops.rope_and_cache(q2, pos, slots, cs, kc, vc, hq, hkv, hd)
    close(q2, q1, rtol=1e-2, atol=1e-2)
    close(kc, kc1, rtol=1e-2, atol=1e-2)
    assert torch.equal(vc, vc1)


@pytest.mark.parametrize("hq,hkv,hd", [(32, 8, 128), (8, 1, 128), (12, 6, 64), (12, 12, 64)])
@pytest.mark.parametrize("lens", [[1], [16, 3], [7, 32, 20], [32] * 5])
def test_prefill_attention_short_prompts_packed(gpu, hq, hkv, hd, lens):
    """Batches of prompts <= 32 / 16 tokens pack 2 / 4 query heads of a GQA group into one
    workgroup: bit-identical to the unpacked kernel and close to the fp32 reference (G = 1:
    no packing)."""
    qkv, *_ = _paged_setup(gpu, lens, hq, hkv, hd, 16)
    cu = torch.tensor([0] + list(np.cumsum(lens)), device=gpu, dtype=torch.int32)
    scale = 1 / math.sqrt(hd)
    old = ops.prefill_set_pack(True)
    try:
        packed = ops.prefill_attention(qkv, cu, max(lens), hq, hkv, hd, scale)
        ops.prefill_set_pack(False)
        plain = ops.prefill_attention(qkv, cu, max(lens), hq, hkv, hd, scale)
    finally:
        ops.prefill_set_pack(old)
    assert torch.equal(packed, plain)
    q, k, v = R.split_qkv(qkv, hq, hkv, hd)
    ref = R.prefill_attention(q, k, v, cu, scale).reshape(len(qkv), -1)
    close(packed, ref, rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("hq,hkv,hd", [(32, 8, 128), (12, 12, 64), (8, 1, 128)])
@pytest.mark.parametrize("lens", [[1], [7, 33, 64], [130, 5]])
def test_prefill_attention(gpu, hq, hkv, hd, lens):
    qkv, *_ = _paged_setup(gpu, lens, hq, hkv, hd, 16)
    cu = torch.tensor([0] + list(np.cumsum(lens)), device=gpu, dtype=torch.int32)
    scale = 1 / math.sqrt(hd)
    out = ops.prefill_attention(qkv, cu, max(lens), hq, hkv, hd, scale)
    q, k, v = R.split_qkv(qkv, hq, hkv, hd)
    ref = R.prefill_attention(q, k, v, cu, scale).reshape(len(qkv), -1)
    close(out, ref, rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("hq,hkv,hd,bs", [(32, 8, 128, 16), (12, 12, 64, 32), (8, 1, 128, 16)])
@pytest.mark.parametrize("lens", [[1, 2, 3], [100, 31, 64, 17], [700, 1025]])
def test_decode_attention_paged(gpu, hq, hkv, hd, bs, lens):
    nblk = sum(-(-n // bs) for n in lens) + 8
    qkv_all, pos, slots, kc, vc, tables = _paged_setup(gpu, lens, hq, hkv, hd, bs, nblk)
    cs = R.rope_cos_sin(2048, hd, 10000.0, device=gpu)
    ops.rope_and_cache(qkv_all, pos, slots, cs, kc, vc, hq, hkv, hd)
    qkv = rnd(len(lens), (hq + 2 * hkv) * hd, dev=gpu)
    ctx = torch.tensor(lens, device=gpu, dtype=torch.int32)
    scale = 1 / math.sqrt(hd)
    q = qkv[:, : hq * hd].reshape(len(lens), hq, hd)
    ref = R.decode_attention(q, kc, vc, tables, ctx, scale).reshape(len(lens), -1)
    # pipelined and one-tile-per-round kernels; the latter unsplit at hd 128 as a workgroup
    # per (sequence, kv head) (small batches, WPI 4) or a wave per item (WPI 1)
    for pipe, wpi in ((1, 0), (0, 4), (0, 1)):
        old = ops.decode_pipelined(pipe)
        old_form = ops.decode_form(wpi)
        try:
            for splits in (1, 2, 4):
                out = ops.decode_attention(qkv, kc, vc, tables, ctx, max(lens), hq, hkv, hd,
                                           scale, num_splits=splits)
                close(out, ref, rtol=2e-2, atol=2e-2)
        finally:
            ops.decode_pipelined(old)
            ops.decode_form(old_form)


@pytest.mark.parametrize("wpi", [1, 4])
@pytest.mark.parametrize("splits", [1, 2, 4])
@pytest.mark.parametrize("hq,hkv", [(32, 8), (8, 1)])
def test_fused_rope_attention(gpu, request, hq, hkv, splits, wpi):
    """dli_decode_attention_fused (split-K QKV reduce + RoPE + KV write + attention in one
    kernel) == linear_rope_cache + decode_attention: the same cache bytes, the same output,
    and the output matches the fp32 reference. splits 1: an unsplit QKV plan (the prologue
    reads the bf16 QKV rows). wpi 1 = a wave per (sequence, kv head), 4 = a
    workgroup per item with the context split over its waves and merged in LDS."""
    old_form = ops.decode_form(wpi)
    request.addfinalizer(lambda: ops.decode_form(old_form))
    hd, bs = 128, 16
    lens = [1, 5, 33, 100, 200, 17, 130]
    B = len(lens)
    nblk = sum(-(-n // bs) for n in lens) + 8
    qkv_all, pos_all, slots_all, kc, vc, tables = _paged_setup(gpu, lens, hq, hkv, hd, bs, nblk)
    cs = R.rope_cos_sin(2048, hd, 500000.0, device=gpu)
    ops.rope_and_cache(qkv_all, pos_all, slots_all, cs, kc, vc, hq, hkv, hd)  # older tokens
    last = torch.tensor(np.cumsum(lens) - 1, device=gpu, dtype=torch.long)
    pos, slots = pos_all[last].contiguous(), slots_all[last].contiguous()
    ctx = torch.tensor(lens, device=gpu, dtype=torch.int32)
    K = 1024
    N = (hq + 2 * hkv) * hd
    x, w = rnd(B, K, dev=gpu), rnd(N, K, dev=gpu, scale=0.05)
    scale = 1 / math.sqrt(hd)
    G.set_plan(B, N, K, "splitk", G.GemmPlan("dli", 0, splits))
    try:
        kc1, vc1 = kc.clone(), vc.clone()
        qkv = ops.linear_rope_cache(x, w, pos, slots, cs, kc1, vc1, hq, hkv, hd)
        ref2 = ops.decode_attention(qkv, kc1, vc1, tables, ctx, max(lens), hq, hkv, hd, scale)
        kc2, vc2 = kc.clone(), vc.clone()
        out = ops.linear_rope_attention(x, w, pos, slots, cs, kc2, vc2, tables, ctx,
                                        max(lens), hq, hkv, hd, scale)
    finally:
        G.clear_plans()
    assert out is not None
    torch.cuda.synchronize()
    assert torch.equal(kc2, kc1) and torch.equal(vc2, vc1)
    close(out, ref2, rtol=1e-2, atol=1e-2)
    # fp32 reference of the whole chain
    qkv_r = R.linear(x, w)
    kc3, vc3 = kc.clone(), vc.clone()
    R.rope_and_cache(qkv_r, pos, slots, cs, kc3, vc3, hq, hkv, hd)
    q = qkv_r[:, : hq * hd].reshape(B, hq, hd)
    ref = R.decode_attention(q, kc3, vc3, tables, ctx, scale).reshape(B, -1)
    close(out, ref, rtol=2e-2, atol=2e-2)


def test_sampling_greedy_and_support(gpu):
    torch.manual_seed(5)
    B, V = 64, 128256
    logits = torch.randn(B, V, device=gpu) * 3
    z = torch.zeros(B, device=gpu)
    ones = torch.ones(B, device=gpu)
    seeds = torch.arange(B, device=gpu, dtype=torch.int64) * 7919
    k1 = torch.ones(B, device=gpu, dtype=torch.int32)
    tok = ops.sample(logits, z, k1, ones, seeds)
    assert torch.equal(tok.long(), logits.argmax(-1))
    temp = torch.full((B,), 0.8, device=gpu)
    topk = torch.full((B,), 50, device=gpu, dtype=torch.int32)
    topp = torch.full((B,), 0.95, device=gpu)
    filt = R.topk_topp_filter(logits, temp, topk, topp)
    for rep in range(4):
        tok = ops.sample(logits, temp, topk, topp, seeds + rep)
        sel = filt.gather(1, tok.long()[:, None]).squeeze(1)
        assert torch.isfinite(sel).all(), "sampled a token outside the top-k/top-p support"


def test_sampling_distribution_matches_reference(gpu):
    """Small vocab, many rows with distinct seeds: empirical frequencies ~ HF probabilities."""
    torch.manual_seed(6)
    V, B = 64, 20000
    row = torch.randn(V, device=gpu) * 2
    logits = row[None].repeat(B, 1).contiguous()
    temp = torch.full((B,), 0.8, device=gpu)
    topk = torch.full((B,), 10, device=gpu, dtype=torch.int32)
    topp = torch.full((B,), 0.9, device=gpu)
    seeds = torch.arange(B, device=gpu, dtype=torch.int64) * 104729 + 11
    tok = ops.sample(logits, temp, topk, topp, seeds)
    p_ref = R.topk_topp_filter(logits[:1], temp[:1], topk[:1], topp[:1]).softmax(-1)[0]
    freq = torch.bincount(tok.long(), minlength=V).float() / B
    assert (freq[p_ref == 0] == 0).all()
    assert (freq - p_ref).abs().max().item() < 0.02


def test_sampling_pure_temperature_gumbel(gpu):
    torch.manual_seed(7)
    V, B = 32, 20000
    row = torch.randn(V, device=gpu)
    logits = row[None].repeat(B, 1).contiguous()
    temp = torch.full((B,), 1.3, device=gpu)
    tok = ops.sample(logits, temp, torch.zeros(B, device=gpu, dtype=torch.int32),
                     torch.ones(B, device=gpu), torch.arange(B, device=gpu, dtype=torch.int64))
    p = (row / 1.3).softmax(-1)
    freq = torch.bincount(tok.long(), minlength=V).float() / B
    assert (freq - p).abs().max().item() < 0.02


@pytest.mark.parametrize("T,E,k", [(1, 8, 2), (37, 8, 2), (300, 4, 2)])
def test_moe_route_and_mlp(gpu, T, E, k):
    torch.manual_seed(8)
    D, F = 256, 512
    x = rnd(T, D, dev=gpu)
    rl = rnd(T, E, dev=gpu)
    w, ids = ops.moe_route(rl, k)
    rw, rids = R.router_topk(rl, k)
    assert torch.equal(ids.long().sort(-1).values, rids.long().sort(-1).values)
    close(w.sort(-1).values, rw.sort(-1).values, rtol=1e-3, atol=1e-3)
    wgu = rnd(E, 2 * F, D, dev=gpu, scale=0.05)
    wd = rnd(E, D, F, dev=gpu, scale=0.05)
    out = ops.moe_mlp(x, wgu, wd, rw, rids)
    ref = R.moe_mlp(x, wgu, wd, rw, rids)
    close(out, ref, rtol=3e-2, atol=3e-2)
    # expert-parallel shard: only experts [2, 4) local
    if E >= 4:
        out2 = ops.moe_mlp(x, wgu[2:4].contiguous(), wd[2:4].contiguous(), rw, rids, 2)
        ref2 = R.moe_mlp(x, wgu[2:4], wd[2:4], rw, rids, 2)
        close(out2, ref2, rtol=3e-2, atol=3e-2)


@pytest.mark.parametrize("tile,splits", [(26, 2), (12, 4), (28, 2), (22, 4)])
def test_moe_down_split_slabs_fused_combine(gpu, tile, splits):
    """Decode-sized MoE whose grouped down projection runs as fp16 split-K slabs reduced
    inside the combine (ops.moe_down_combine) == the fp32 reference, and == the unfused
    path (GEMM with the bf16 y, then the combine) within bf16 rounding; the experts' rows
    are uneven (seeded multinomial routing) and one expert gets no row."""
    torch.manual_seed(21)
    T, E, k, D, F = 96, 8, 2, 512, 1024
    x = rnd(T, D, dev=gpu)
    logits = rnd(T, E, dev=gpu)
    logits[:, 5] = -30.0                          # expert 5 is never picked
    rw, rids = R.router_topk(logits, k)
    wgu = rnd(E, 2 * F, D, dev=gpu, scale=0.05)
    wd = rnd(E, D, F, dev=gpu, scale=0.05)
    key = (G._bucket(T * k), D, F, "none", E)
    old = G._grouped_cache.get(key)
    G._grouped_cache[key] = G.GemmPlan("dli", tile, splits)
    try:
        assert ops.moe_slab_plan(G.grouped_plan(T * k, D, F, "none", E))
        out = ops.moe_mlp(x, wgu, wd, rw, rids)
        G._grouped_cache[key] = G.GemmPlan("dli", tile, 1)
        unfused = ops.moe_mlp(x, wgu, wd, rw, rids)
    finally:
        if old is None:
            G._grouped_cache.pop(key, None)
        else:
            G._grouped_cache[key] = old
    ref = R.moe_mlp(x, wgu, wd, rw, rids)
    close(out, ref, rtol=3e-2, atol=3e-2)
    close(out, unfused, rtol=2e-2, atol=2e-2)


def test_sampling_fallback_path_adversarial(gpu):
    """Top-k values concentrated in ONE thread's strided slice force the exact radix-select
    fallback (the register top-8 fast path cannot prove completeness)."""
    torch.manual_seed(9)
    B, V = 4, 128256
    logits = torch.randn(B, V, device=gpu)
    logits[:, 0::512][:, :60] += 20.0            # 60 huge values all owned by thread 0
    temp = torch.full((B,), 0.8, device=gpu)
    topk = torch.full((B,), 50, device=gpu, dtype=torch.int32)
    topp = torch.full((B,), 0.95, device=gpu)
    filt = R.topk_topp_filter(logits, temp, topk, topp)
    for rep in range(8):
        tok = ops.sample(logits, temp, topk, topp,
                         torch.arange(B, device=gpu, dtype=torch.int64) + 1000 * rep)
        assert torch.isfinite(filt.gather(1, tok.long()[:, None])).all()
        assert (tok % 512 == 0).all()


@pytest.mark.parametrize("B,V", [(64, 128256), (512, 128256)])
def test_sampling_two_phase_large_batch(gpu, B, V):
    """The two-phase sampler with its batch limit raised (dli_sample_set_split_max_b, the
    DLI_SAMPLE_SPLIT_MAX_B A/B switch): 32 chunks per 128k row, same tokens as one phase."""
    lib = ops.N.require_native()
    old = lib.dli_sample_set_split_max_b(512)
    ops._sample_wss.clear()
    try:
        torch.manual_seed(16)
        logits = torch.randn(B, V, device=gpu) * 3
        ws = ops._sample_ws(logits.device, B, V)
        assert ws is not None
        for T, K, P in [(0.8, 50, 0.95), (0.0, 1, 1.0), (1.0, 64, 0.5)]:
            temp = torch.full((B,), T, device=gpu)
            topk = torch.full((B,), K, device=gpu, dtype=torch.int32)
            topp = torch.full((B,), P, device=gpu)
            seeds = torch.arange(B, device=gpu, dtype=torch.int64) * 7919 + 5
            one = torch.empty(B, dtype=torch.int32, device=gpu)
            two = torch.empty(B, dtype=torch.int32, device=gpu)
            for o, w in ((one, None), (two, ws)):
                assert lib.dli_sample(ops._p(o), ops._p(logits), logits.stride(0), B, V,
                                      ops._p(temp), ops._p(topk), ops._p(topp), ops._p(seeds),
                                      ops._p(w), ops._st()) == 0
            assert torch.equal(one, two), (T, K, P)
        torch.cuda.synchronize()
    finally:
        lib.dli_sample_set_split_max_b(old)
        ops._sample_wss.clear()


@pytest.mark.parametrize("B,V", [(1, 128256), (3, 50257), (8, 128256), (2, 1000)])
def test_sampling_two_phase_matches_one_phase(gpu, B, V):
    """Small batches sample in two phases (per-chunk candidate lists, sampling.hip
    sample_chunk_kernel): the same tokens as the one-workgroup-per-row kernel for every
    parameter mix — greedy, top-k 1 / 50 / 64 with top-p, top-k 100 and top-k 0 (full-row
    paths) — and for rows whose chunks overflow their candidate slots (a tie-heavy row)."""
    torch.manual_seed(15)
    logits = torch.randn(B, V, device=gpu) * 3
    if B >= 2:                                 # 300 ties above everything else in one
        logits[1, V // 3:V // 3 + 300] = 30.0  # chunk: it overflows -> full-row path (a
        # whole row of ties is not used: the one-phase kernel keeps an arbitrary 2048 of them)
    lib = ops.N.require_native()
    ws = ops._sample_ws(logits.device, B, V)
    assert ws is not None
    ones = torch.ones(B, device=gpu)
    for T, K, P in [(0.0, 1, 1.0), (0.8, 1, 1.0), (0.8, 50, 0.95), (1.0, 64, 0.5),
                    (0.7, 100, 0.9), (1.1, 0, 0.9), (0.9, 0, 1.0), (0.8, 5, 1.0)]:
        temp = torch.full((B,), T, device=gpu)
        topk = torch.full((B,), K, device=gpu, dtype=torch.int32)
        topp = ones * P
        for rep in range(3):
            seeds = torch.arange(B, device=gpu, dtype=torch.int64) * 7919 + 31 * rep
            one = torch.empty(B, dtype=torch.int32, device=gpu)
            two = torch.empty(B, dtype=torch.int32, device=gpu)
            for o, w in ((one, None), (two, ws)):
                rc = lib.dli_sample(ops._p(o), ops._p(logits), logits.stride(0), B, V,
                                    ops._p(temp), ops._p(topk), ops._p(topp), ops._p(seeds),
                                    ops._p(w), ops._st())
                assert rc == 0
            assert torch.equal(one, two), (T, K, P, one, two)
    torch.cuda.synchronize()
    assert int(ws[:32].view(torch.int32).abs().sum()) == 0        # overflow flags reset


@pytest.mark.parametrize("epi", ["none", "silu_mul"])
def test_grouped_8phase_rows_bound(gpu, epi):
    """Grouped tile 22 with M = the largest group's rows (the MoE prefill launch) over groups
    of 0 / 300 / 1029 / 513 rows: row tiles past a group's end are skipped, partial ones
    clamped."""
    torch.manual_seed(14)
    sizes = [0, 300, 1029, 513]
    E, N, K = len(sizes), 512, 640
    x = rnd(sum(sizes), K, dev=gpu)
    w = rnd(E, N, K, dev=gpu, scale=0.05)
    off = torch.tensor([0] + list(__import__("itertools").accumulate(sizes)), dtype=torch.int32,
                       device=gpu)
    refs = []
    for e in range(E):
        y = R.linear(x[off[e]:off[e + 1]], w[e])
        refs.append(R.silu_mul(y.float().to(BF)) if epi == "silu_mul" else y)
    out = ops._gemm_native(x, w, epi, plan=G.GemmPlan("dli", 22, 1), groups=E, group_off=off,
                           rows_per_group=max(sizes))
    close(out, torch.cat(refs), rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("epi", ["none", "silu_mul"])
def test_grouped_gemm_all_tiles_and_splitk(gpu, epi):
    """Grouped (MoE) GEMM over uneven groups (one empty, one past a 128-row tile) for every
    tile id and split-K factor, against per-group fp32 references."""
    torch.manual_seed(12)
    sizes = [0, 37, 170, 5]
    E, N, K = len(sizes), 256, 1024
    rows = sum(sizes)
    x = rnd(rows, K, dev=gpu)
    w = rnd(E, N, K, dev=gpu, scale=0.05)
    off = torch.tensor([0] + list(__import__("itertools").accumulate(sizes)), dtype=torch.int32,
                       device=gpu)
    refs = []
    for e in range(E):
        xe = x[off[e]:off[e + 1]]
        y = R.linear(xe, w[e])
        refs.append(R.silu_mul(y.float().to(BF)) if epi == "silu_mul" else y)
    ref = torch.cat(refs)
    for tile in G.TILES:
        if not G.tile_ok(tile, epi) or tile == 55:         # 55 (persistent): no grouped mode
            continue
        for splits in (1, 2, 4):
            out = ops._gemm_native(x, w, epi, plan=G.GemmPlan("dli", tile, splits), groups=E,
                                   group_off=off, rows_per_group=rows)
            close(out, ref, rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("tile", [22, 45])
def test_moe_mlp_prefill_grouped_path(gpu, monkeypatch, tile):
    """Prefill-sized MoE (rows per expert above the threshold) takes the grouped 256x256
    path (grid bounded by the largest expert's rows) on the 8-phase (22) or the two-barrier
    4-wave tile (45, the default); same result as the reference."""
    monkeypatch.setattr(ops, "_MOE_PREFILL_ROWS", 16)
    monkeypatch.setattr(ops.G, "MOE_PREFILL_TILE", tile)
    torch.manual_seed(13)
    T, E, k, D, F = 200, 4, 2, 256, 512
    x = rnd(T, D, dev=gpu)
    rw, rids = R.router_topk(rnd(T, E, dev=gpu), k)
    wgu = rnd(E, 2 * F, D, dev=gpu, scale=0.05)
    wd = rnd(E, D, F, dev=gpu, scale=0.05)
    close(ops.moe_mlp(x, wgu, wd, rw, rids), R.moe_mlp(x, wgu, wd, rw, rids),
          rtol=3e-2, atol=3e-2)


def test_vocab_parallel_candidates_sample_like_full_vocab(gpu):
    """Vocab-parallel head: per-slice top-64 candidates (ascending ids) merged on rank 0 and
    sampled with the same seeds give the same tokens as sampling the full vocabulary."""
    torch.manual_seed(14)
    B, D, V, N = 64, 256, 8000, 4
    h = rnd(B, D, dev=gpu)
    w = rnd(V, D, dev=gpu, scale=0.2)
    full = ops.linear(h, w, epi=ops.HEAD_EPI)                # the single-stage head's logits
    bounds = [round(i * V / N) for i in range(N + 1)]
    vals, ids = zip(*[ops.head_candidates(h, w[bounds[r]:bounds[r + 1]].contiguous(), bounds[r],
                                          64) for r in range(N)])
    vals, ids = torch.cat(vals, 1), torch.cat(ids, 1)
    assert torch.all(ids[:, 1:] > ids[:, :-1])                # ascending token ids
    temp = torch.full((B,), 0.8, device=gpu)
    topk = torch.full((B,), 50, device=gpu, dtype=torch.int32)
    topk[::7] = 1                                             # some greedy rows
    topp = torch.full((B,), 0.95, device=gpu)
    seeds = torch.arange(B, device=gpu, dtype=torch.int64) * 7919 + 11
    a = ops.sample(full, temp, topk, topp, seeds)
    b = ops.sample(vals, temp, topk, topp, seeds, ids=ids)
    assert torch.equal(a, b)


def test_feed_ids(gpu):
    """Lookahead id feed: ids[i] = feed[src[i]] where src[i] >= 0, host ids elsewhere."""
    ids = torch.arange(100, 164, device=gpu, dtype=torch.int32)
    feed = torch.arange(5000, 5040, device=gpu, dtype=torch.int32)
    src = torch.full((64,), -1, device=gpu, dtype=torch.int32)
    src[::3] = torch.arange(0, 64, 3, device=gpu, dtype=torch.int32) % 40
    ref = torch.where(src >= 0, feed[src.clamp(min=0).long()], ids)
    ops.feed_ids(ids, src, feed)
    assert torch.equal(ids, ref)


@pytest.mark.parametrize("T,E,k", [(5, 64, 2), (129, 16, 4), (64, 8, 8)])
def test_moe_route_wide(gpu, T, E, k):
    """Wave-per-token router at the E <= 64 limit, k up to E (HF: lowest index on ties)."""
    torch.manual_seed(9)
    rl = rnd(T, E, dev=gpu)
    rl[0] = 0                                   # all-tie row: experts 0..k-1, weights 1/k
    w, ids = ops.moe_route(rl, k)
    rw, rids = R.router_topk(rl, k)
    assert torch.equal(ids[1:].long().sort(-1).values, rids[1:].long().sort(-1).values)
    assert ids[0].tolist() == list(range(k))
    close(w.sort(-1).values, rw.sort(-1).values, rtol=1e-3, atol=1e-3)
    assert torch.allclose(w.sum(-1), torch.ones(T, device=gpu), atol=1e-5)


@pytest.mark.parametrize("T,E,D", [(1, 8, 4096), (37, 8, 256), (512, 8, 4096), (64, 4, 512),
                                   (9, 2, 128)])
def test_moe_router_fused(gpu, T, E, D):
    """The fused gate (moe_router_kernel: E <= 8 dot products per token, bf16 logits, softmax,
    top-2, renormalise) against an fp32 reference: the picks are the top-2 of the bf16-rounded
    logits up to near-ties (summation order may move a logit by one bf16 ulp), distinct per
    token, and the weights are the renormalised softmax of the picked logits."""
    torch.manual_seed(41)
    k = 2
    h = rnd(T, D, dev=gpu)
    wr = rnd(E, D, dev=gpu, scale=0.05)
    w, ids = ops.moe_router(h, wr, k)
    lb = (h.float() @ wr.float().t()).to(BF).float()
    il = ids.long()
    assert ((il >= 0) & (il < E)).all() and (il[:, 0] != il[:, 1]).all()
    kth = lb.topk(k, -1).values[:, -1:]
    tol = 2 ** -7 * lb.abs().amax(-1, keepdim=True)
    assert (lb.gather(1, il) >= kth - tol).all()
    p = lb.softmax(-1).gather(1, il)
    close(w, p / p.sum(-1, keepdim=True), rtol=2e-2, atol=2e-3)
    assert torch.allclose(w.sum(-1), torch.ones(T, device=gpu), atol=1e-5)


@pytest.mark.parametrize("M,splits", [(512, 4), (37, 2), (5, 8)])
def test_add_rmsnorm_with_fused_gate(gpu, M, splits):
    """The Mixtral O-projection reduce with the MoE gate inside (dli_splitk_add_rmsnorm_route)
    == the plain reduce followed by moe_router: the same output rows and residual bit for
    bit, the same picks up to one-ulp near-ties of the bf16 logits, the same weights."""
    torch.manual_seed(43)
    K = N = 4096
    x, w = rnd(M, K, dev=gpu), rnd(N, K, dev=gpu, scale=0.02)
    r0, nw = rnd(M, N, dev=gpu), (1.0 + 0.1 * rnd(N, dev=gpu)).to(BF)
    wr = rnd(8, N, dev=gpu, scale=0.05)
    p = G.GemmPlan("dli", 28, splits)
    assert p.tile in G.SLAB16_TILES
    r1, r2 = r0.clone(), r0.clone()
    o1, tw1, ti1 = ops.linear_add_rmsnorm(x, w, r1, nw, 1e-5, plan=p, route=(wr, 2))
    o2 = ops.linear_add_rmsnorm(x, w, r2, nw, 1e-5, plan=p)
    tw2, ti2 = ops.moe_router(o2, wr, 2)
    assert torch.equal(o1, o2) and torch.equal(r1, r2)
    lb = (o2.float() @ wr.float().t()).to(BF).float()
    kth = lb.topk(2, -1).values[:, -1:]
    tol = 2 ** -7 * lb.abs().amax(-1, keepdim=True)
    assert (lb.gather(1, ti1.long()) >= kth - tol).all()
    same = (ti1 == ti2).all(-1)
    assert same.float().mean() > 0.95
    close(tw1[same], tw2[same], rtol=1e-2, atol=1e-3)


@pytest.mark.parametrize("splits", [2, 4])
def test_moe_combine_fused_with_next_norm(gpu, splits):
    """A decode MoE layer's deferred combine (ops.MoEPending) run inside the next layer's
    add + RMSNorm (dli_moe_combine_add_rmsnorm) == the plain combine, then the add + RMSNorm
    kernel: the residual bit for bit, the normalised rows within one bf16 ulp (the row sum of
    squares is reduced in another order); and the residual-only form of a last layer."""
    torch.manual_seed(47)
    T, E, k, D, F = 96, 8, 2, 4096, 512
    x = rnd(T, D, dev=gpu)
    logits = rnd(T, E, dev=gpu)
    logits[:, 5] = -30.0                          # expert 5 is never picked
    rw, rids = R.router_topk(logits, k)
    wgu = rnd(E, 2 * F, D, dev=gpu, scale=0.05)
    wd = rnd(E, D, F, dev=gpu, scale=0.05)
    key = (G._bucket(T * k), D, F, "none", E)
    old = G._grouped_cache.get(key)
    G._grouped_cache[key] = G.GemmPlan("dli", 12, splits)
    try:
        pend = ops.moe_mlp(x, wgu, wd, rw, rids, defer_combine=True)
        assert isinstance(pend, ops.MoEPending)
        r0, nw = rnd(T, D, dev=gpu), (1.0 + 0.1 * rnd(D, dev=gpu)).to(BF)
        r1, r2, r3 = r0.clone(), r0.clone(), r0.clone()
        plain = pend.materialize()
        close(plain, R.moe_mlp(x, wgu, wd, rw, rids), rtol=3e-2, atol=3e-2)
        out_b = ops.add_rmsnorm(plain, r2, nw, 1e-5)
        out_a = ops.add_rmsnorm(pend, r1, nw, 1e-5)
        assert torch.equal(r1, r2)
        close(out_a, out_b, rtol=1e-2, atol=1e-2)
        assert pend.add_rmsnorm(r3, None, 1e-5) is None
        assert torch.equal(r3, r2)
    finally:
        if old is None:
            G._grouped_cache.pop(key, None)
        else:
            G._grouped_cache[key] = old


@pytest.mark.parametrize("tile", [12, 2, 10, 17])
def test_grouped_gate_up_reads_rows_through_permutation(gpu, tile):
    """dli_gemm_grouped_gather (the MoE gate/up without the gathered copy of its input) ==
    the grouped SiLU*up GEMM of the gathered rows, bit for bit: same tile, same sums, only
    the A-row addresses differ; uneven groups incl. an empty one and one past a tile."""
    torch.manual_seed(53)
    T, E, D, F2 = 150, 4, 512, 1024
    sizes = [37, 0, 190, 73]
    rows = sum(sizes)
    x = rnd(T, D, dev=gpu)
    src = torch.randint(0, T, (rows,), dtype=torch.int32, device=gpu)
    off = torch.tensor([0] + list(__import__("itertools").accumulate(sizes)), dtype=torch.int32,
                       device=gpu)
    w = rnd(E, F2, D, dev=gpu, scale=0.05)
    if not G.tile_ok(tile, "silu_mul"):
        pytest.skip("tile without the SiLU pairing")
    ref = ops._gemm_native(x[src.long()].contiguous(), w, "silu_mul",
                           plan=G.GemmPlan("dli", tile, 1), groups=E, group_off=off,
                           rows_per_group=rows)
    out = torch.full((rows, F2 // 2), float("nan"), dtype=BF, device=gpu)
    ops._native_call("dli_gemm_grouped_gather", ops._p(x), x.stride(0), ops._p(w), w.stride(-2),
                     ops._p(out), out.stride(0), rows, F2, D, tile, ops._p(src), ops._p(off), E,
                     ops._st())
    assert torch.equal(out, ref)


@pytest.mark.parametrize("S,V,c", [(37, 16032, 64), (5, 4008, 64), (3, 64, 64), (9, 50257, 50)])
def test_topk_rows_kernel(gpu, S, V, c):
    """HIP per-row top-c (vocab-parallel head candidates) vs torch.topk: same value multiset,
    ids ascending and offset, every value above the c-th largest present, ties broken to the
    lowest index; exercised on continuous and heavily tied rows."""
    from distributed_llm_inferencing_amd.ops import _native
    torch.manual_seed(3)
    off = 1000
    for tied in (False, True):
        x = torch.randn(S, V, device=gpu)
        if tied:
            x = (x * 2).round() / 2                 # few distinct values: many ties at the cut
        v = torch.empty(S, c, device=gpu)
        i = torch.empty(S, c, dtype=torch.int32, device=gpu)
        _native.call("dli_topk_rows", v.data_ptr(), i.data_ptr(), x.data_ptr(), x.stride(0), S,
                     V, c, off, torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        ref = torch.topk(x, c, dim=-1).values
        assert torch.equal(v.sort(-1, descending=True).values, ref)
        assert bool((i[:, 1:] > i[:, :-1]).all())                  # ascending ids
        loc = (i - off).long()
        assert torch.equal(x.gather(1, loc), v)                     # ids point at values
        kth = ref[:, -1:]
        assert torch.equal((x > kth).sum(-1), (v > kth).sum(-1))    # all strictly larger
        for r in range(S):                                          # ties: lowest indices
            eq = (x[r] == kth[r]).nonzero().flatten()
            need = int((v[r] == kth[r]).sum())
            assert torch.equal(loc[r][v[r] == kth[r]], eq[:need])


def test_head_candidates_native_matches_reference(gpu):
    torch.manual_seed(4)
    h = rnd(19, 256, dev=gpu)
    w = rnd(3000, 256, dev=gpu, scale=0.1)
    v, i = ops.head_candidates(h, w, 5000, 64)
    lg = ops.linear(h, w, epi=ops.HEAD_EPI).float()    # same logits the op ranks
    # ties (frequent in bf16) go to the lower token id: a stable descending sort
    rv, ri = torch.sort(lg, dim=-1, descending=True, stable=True)
    rv, ri = rv[:, :64], ri[:, :64]
    ri, perm = torch.sort((ri + 5000).to(torch.int32), dim=-1)
    assert torch.equal(i, ri)
    assert torch.equal(v, rv.gather(1, perm))
    close(v, R.linear(h, w, out_dtype=torch.float32).gather(1, (i - 5000).long()),
          rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("B,V", [(512, 128256), (7, 32000), (3, 50257), (64, 1000)])
def test_sampler_bf16_logits_equal_fp32_upcast(gpu, B, V):
    """The sampler reads bf16 logits (the LM head in the model dtype, as HF's
    ``lm_head(h).float()``) and compares their exact fp32 values: every token equals
    sampling the fp32 upcast of the same logits — greedy, top-k/top-p, plain temperature,
    the one- and the two-phase (small-batch) paths."""
    torch.manual_seed(22)
    lg = (torch.randn(B, V, device=gpu) * 3).to(BF)
    temp = torch.full((B,), 0.8, device=gpu)
    topk = torch.full((B,), 50, device=gpu, dtype=torch.int32)
    topp = torch.full((B,), 0.95, device=gpu)
    topk[1::5] = 1                                            # greedy rows
    topk[2::5] = 0                                            # top-p over the whole row
    temp[3::5] = 0.0                                          # greedy by temperature
    topp[4::5] = 1.0
    seeds = torch.arange(B, device=gpu, dtype=torch.int64) * 104729 + 3
    a = ops.sample(lg, temp, topk, topp, seeds)
    b = ops.sample(lg.float(), temp, topk, topp, seeds)
    assert torch.equal(a, b)


def test_topk_rows_bf16(gpu):
    from distributed_llm_inferencing_amd.ops import _native
    torch.manual_seed(5)
    S, V, c = 11, 16000, 64
    x = (torch.randn(S, V, device=gpu)).to(BF)               # bf16: many ties
    st = torch.cuda.current_stream().cuda_stream
    out = []
    for t in (x, x.float()):
        v = torch.empty(S, c, device=gpu)
        i = torch.empty(S, c, dtype=torch.int32, device=gpu)
        fn = "dli_topk_rows_bf16" if t.dtype == BF else "dli_topk_rows"
        _native.call(fn, v.data_ptr(), i.data_ptr(), t.data_ptr(), t.stride(0), S, V, c, 7, st)
        out.append((v, i))
    torch.cuda.synchronize()
    assert torch.equal(out[0][0], out[1][0]) and torch.equal(out[0][1], out[1][1])


def test_ep_pack_and_combine(gpu):
    """Expert-parallel dispatch pack (fixed-capacity buckets) and the weighted combine:
    every (token, pick) row lands in its destination's bucket with its expert id, unused
    rows keep -1, and combining the returned rows equals the fp32 reference sum."""
    torch.manual_seed(15)
    T, k, D, N, e_per = 300, 2, 512, 4, 2
    x = rnd(T, D, dev=gpu)
    _w, ids = R.router_topk(rnd(T, N * e_per, dev=gpu), k)
    ids = ids.to(torch.int32)
    C = T * min(k, e_per)
    base = torch.arange(N, dtype=torch.int32, device=gpu) * C
    sx, se, pos = ops.ep_pack(x, ids, e_per, base, N * C)
    torch.cuda.synchronize()
    p = pos.long()
    assert torch.equal(se[p.flatten()], ids.flatten())
    assert torch.equal(sx[p.flatten()], x.repeat_interleave(k, 0))
    dest = (ids.long() // e_per)
    assert bool(((p >= dest * C) & (p < dest * C + C)).all())          # inside its bucket
    assert int((se >= 0).sum()) == T * k and len(set(p.flatten().tolist())) == T * k
    y = rnd(N * C, D, dev=gpu)
    w = torch.rand(T, k, device=gpu)
    out = ops.moe_combine(y, w, pos)
    ref = (y[p].float() * w.unsqueeze(-1)).sum(1)
    close(out, ref, rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("lens,hq,hkv", [([2048, 300], 32, 8), ([8192], 8, 2),
                                          ([1000, 400, 5, 700], 32, 8)])
def test_prefill_attention_long(gpu, lens, hq, hkv):
    """Long prompts: 2k and 8k-token causal GQA prefill vs the fp32
    reference (the 8k case with fewer heads so the fp32 reference's score matrix fits)."""
    torch.manual_seed(21)
    hd = 128
    T = sum(lens)
    qkv = rnd(T, (hq + 2 * hkv) * hd, dev=gpu)
    cu = torch.tensor([0] + list(np.cumsum(lens)), device=gpu, dtype=torch.int32)
    scale = 1 / math.sqrt(hd)
    q, k, v = R.split_qkv(qkv, hq, hkv, hd)
    ref = R.prefill_attention(q, k, v, cu, scale).reshape(T, -1)
    for thr in (1, 1 << 30):            # the 256-row 32x32x16 kernel and the 64-row kernel
        old = ops.prefill_long_min_len(thr)
        try:
            out = ops.prefill_attention(qkv, cu, max(lens), hq, hkv, hd, scale)
        finally:
            ops.prefill_long_min_len(old)
        close(out, ref, rtol=2e-2, atol=2e-2)


def test_decode_attention_32k_context(gpu):
    """Decode against a 32k-token paged context (and a short one in the same batch), with
    the default split heuristic and forced splits."""
    torch.manual_seed(22)
    hq, hkv, hd, bs = 32, 8, 128, 16
    lens = [32768, 77]
    nblk = sum(-(-n // bs) for n in lens) + 4
    kc = rnd(nblk, hkv, bs, hd, dev=gpu)
    vc = rnd(nblk, hkv, bs, hd, dev=gpu)
    perm = torch.randperm(nblk - 4, device=gpu).to(torch.int32)      # scattered blocks
    maxb = -(-max(lens) // bs)
    tables, o = [], 0
    for n in lens:
        nb = -(-n // bs)
        tables.append(torch.cat([perm[o:o + nb], torch.zeros(maxb - nb, dtype=torch.int32,
                                                               device=gpu)]))
        o += nb
    tables = torch.stack(tables)
    qkv = rnd(len(lens), (hq + 2 * hkv) * hd, dev=gpu)
    ctx = torch.tensor(lens, device=gpu, dtype=torch.int32)
    scale = 1 / math.sqrt(hd)
    q = qkv[:, : hq * hd].reshape(len(lens), hq, hd)
    ref = R.decode_attention(q, kc, vc, tables, ctx, scale).reshape(len(lens), -1)
    for pipe in (1, 0):                      # pipelined and one-tile-per-round kernels
        old = ops.decode_pipelined(pipe)
        try:
            for splits in (None, 8, 32):
                out = ops.decode_attention(qkv, kc, vc, tables, ctx, max(lens), hq, hkv, hd,
                                           scale, num_splits=splits)
                close(out, ref, rtol=2e-2, atol=2e-2)
        finally:
            ops.decode_pipelined(old)


@pytest.mark.parametrize("hq,hkv,hd,bs,chunks", [
    (32, 8, 128, 16, [(100, 37), (2053, 512), (16, 16), (1, 1)]),
    (12, 12, 64, 32, [(70, 70), (300, 64), (129, 1)]),
    (8, 1, 128, 16, [(4096, 700)]),
    # short chunks only: the head-packed kernel over a paged cache
    (32, 8, 128, 16, [(100, 17), (33, 32), (5, 5)]),
    (8, 2, 128, 16, [(64, 16), (300, 9)])])
def test_prefill_attention_paged_chunks(gpu, hq, hkv, hd, bs, chunks):
    """Chunked prefill: each chunk of queries (positions [ctx-L, ctx)) attends over all ctx
    keys of its sequence in a scattered paged cache, vs the fp32 reference."""
    torch.manual_seed(23)
    ctxs = [c for c, _ in chunks]
    lens = [n for _, n in chunks]
    nblk = sum(-(-c // bs) for c in ctxs) + 4
    kc = rnd(nblk, hkv, bs, hd, dev=gpu)
    vc = rnd(nblk, hkv, bs, hd, dev=gpu)
    perm = torch.randperm(nblk - 4, device=gpu).to(torch.int32)
    maxb = -(-max(ctxs) // bs)
    tables, o = [], 0
    for c in ctxs:
        nb = -(-c // bs)
        tables.append(torch.cat([perm[o:o + nb], torch.zeros(maxb - nb, dtype=torch.int32,
                                                               device=gpu)]))
        o += nb
    tables = torch.stack(tables)
    T = sum(lens)
    qkv = rnd(T, (hq + 2 * hkv) * hd, dev=gpu)
    cu = torch.tensor([0] + list(np.cumsum(lens)), device=gpu, dtype=torch.int32)
    ctx = torch.tensor(ctxs, device=gpu, dtype=torch.int32)
    scale = 1 / math.sqrt(hd)
    out = ops.prefill_attention_paged(qkv, cu, max(lens), ctx, tables, kc, vc, hq, hkv, hd,
                                      scale)
    q = qkv[:, : hq * hd].reshape(T, hq, hd)
    ref = R.prefill_attention_paged(q, kc, vc, cu, ctx, tables, scale).reshape(T, -1)
    close(out, ref, rtol=2e-2, atol=2e-2)


def test_rccl_comm_module_self_exchange(gpu):
    """csrc/runtime/comm.cpp on one GPU: a world-1 communicator, send-to-self + receive in one
    group on the current stream (the pipeline data plane's DLI_PP_COMM=rccl path), several
    buffers of different sizes in one group, then an invalid peer fails loudly."""
    from distributed_llm_inferencing_amd.runtime import RcclComm
    assert RcclComm.available()
    comm = RcclComm(RcclComm.unique_id(), 1, 0)
    st = torch.cuda.current_stream().cuda_stream
    a = torch.randn(4096, 512, device=gpu).to(BF)
    b = torch.arange(1000, device=gpu, dtype=torch.int32)
    ra, rb = torch.empty_like(a), torch.empty_like(b)
    comm.exchange([(a, 0), (b, 0)], [(ra, 0), (rb, 0)], st)
    torch.cuda.synchronize()
    assert torch.equal(ra, a) and torch.equal(rb, b)
    with pytest.raises(RuntimeError):
        comm.exchange([(a, 3)], [], st)
    comm.close()
