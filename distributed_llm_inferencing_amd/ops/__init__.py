"""Op API used by the models. CUDA(HIP) tensors -> gfx950 kernels; CPU tensors -> PyTorch
reference (``ops/reference.py``). There is no silent fallback on a GPU: if the kernel
library is missing, the first GPU op raises (``_native.require_native``).

All functions take/return torch tensors and launch on torch's current stream.
"""
from __future__ import annotations

import math
import time
from typing import Optional

import torch

from . import _native as N
from . import gemm as G
from . import reference as R

_native_call = N.call
_p = N.ptr
# rows per expert from which eager (prefill) MoE GEMMs take the grouped 256x256 tile
_MOE_PREFILL_ROWS = 1024


def _use_native(t: torch.Tensor) -> bool:
    """GPU tensors always run the HIP kernels (no switch reroutes them to torch ops)."""
    return t.is_cuda


def _st():
    return N.stream_ptr()


# ----------------------------------------------------------------------------- norms
def rmsnorm(x, w, eps, residual_copy: Optional[torch.Tensor] = None):
    """out = rmsnorm(x)*w; if residual_copy is given it receives a copy of x."""
    if not _use_native(x):
        if residual_copy is not None:
            residual_copy.copy_(x)
        return R.rmsnorm(x, w, eps)
    out = torch.empty_like(x)
    rows, dim = x.shape
    _native_call("dli_rmsnorm", _p(out), _p(residual_copy), _p(x), _p(w), rows, dim, eps, _st())
    return out


def add_rmsnorm(x, residual, w, eps):
    """residual += x (in place); returns rmsnorm(residual)*w. ``x`` may be a ``MoEPending``
    (a MoE layer's output not yet combined): the combine, the add and the norm then run as
    one kernel."""
    if isinstance(x, MoEPending):
        return x.add_rmsnorm(residual, w, eps)
    if not _use_native(x):
        out, r = R.fused_add_rmsnorm(x, residual, w, eps)
        residual.copy_(r)
        return out
    out = torch.empty_like(x)
    rows, dim = x.shape
    _native_call("dli_fused_add_rmsnorm", _p(out), _p(residual), _p(x), _p(w), rows, dim, eps,
                 _st())
    return out


def layernorm(x, w, b, eps, residual_copy: Optional[torch.Tensor] = None):
    if not _use_native(x):
        if residual_copy is not None:
            residual_copy.copy_(x)
        return R.layernorm(x, w, b, eps)
    out = torch.empty_like(x)
    rows, dim = x.shape
    _native_call("dli_layernorm", _p(out), _p(residual_copy), _p(x), _p(w), _p(b), rows, dim,
                 eps, _st())
    return out


def add_layernorm(x, residual, w, b, eps):
    if not _use_native(x):
        out, r = R.fused_add_layernorm(x, residual, w, b, eps)
        residual.copy_(r)
        return out
    out = torch.empty_like(x)
    rows, dim = x.shape
    _native_call("dli_fused_add_layernorm", _p(out), _p(residual), _p(x), _p(w), _p(b), rows,
                 dim, eps, _st())
    return out


class MoEPending:
    """A decode MoE layer's output before its combine: the grouped down projection's fp16
    split-K slabs, the routing weights and the row of each (token, pick). ``add_rmsnorm``
    (the next layer's input norm, via ``ops.add_rmsnorm``) combines, adds into the residual
    and normalises in one kernel (``dli_moe_combine_add_rmsnorm``); ``materialize()`` runs
    the plain combine for any other consumer. The slab workspace must not be reused before
    the consumer has run (the next GEMM to use it is the next layer's)."""

    def __init__(self, ws, splits: int, rows: int, topk_w, pos, shape, dtype, device):
        self.ws, self.splits, self.rows = ws, splits, rows
        self.topk_w, self.pos = topk_w, pos
        self.shape, self.dtype, self.device = shape, dtype, device

    def materialize(self) -> torch.Tensor:
        T, D = self.shape
        out = torch.empty(T, D, dtype=self.dtype, device=self.device)
        k = self.topk_w.shape[1]
        _native_call("dli_moe_combine_slabs", _p(out), _p(self.ws), self.splits, self.rows,
                     _p(self.topk_w), _p(self.pos), T, k, D, _st())
        return out

    def add_rmsnorm(self, residual, w, eps):
        """w None: the residual add only (a stage's last layer); returns None then."""
        T, D = self.shape
        if D != 4096 or not residual.is_contiguous():
            m = self.materialize()
            if w is None:
                residual.add_(m)
                return None
            return add_rmsnorm(m, residual, w, eps)
        out = torch.empty(T, D, dtype=self.dtype, device=self.device) if w is not None else None
        k = self.topk_w.shape[1]
        _native_call("dli_moe_combine_add_rmsnorm", _p(out), _p(residual), _p(self.ws),
                     self.splits, self.rows, _p(self.topk_w), _p(self.pos), T, k, D, _p(w),
                     float(eps), _st())
        return out


class NormedRows:
    """rmsnorm(residual) * w, not yet computed: batch-1 decode (models/model.py) hands this to
    the consuming GEMV, whose prologue normalises the rows into LDS (``dli_gemv_fused``), so
    the O / down projections add straight into the residual (``linear_residual``) and no
    reduce + norm kernel runs between them. Consumers without such a prologue call
    ``materialize()``. The residual must not change before the consumer has run."""
    __slots__ = ("residual", "w", "eps")

    def __init__(self, residual: torch.Tensor, w: torch.Tensor, eps: float):
        self.residual, self.w, self.eps = residual, w, eps

    @property
    def shape(self):
        return self.residual.shape

    @property
    def device(self):
        return self.residual.device

    @property
    def dtype(self):
        return self.residual.dtype

    def materialize(self) -> torch.Tensor:
        return rmsnorm(self.residual, self.w, self.eps)


def deferred_norm_ok(x: torch.Tensor) -> bool:
    """Whether a decode step of ``x.shape[0]`` rows runs the reduce-free GEMV chain."""
    M, K = x.shape
    return (G.DEFER_NORM and _use_native(x) and M <= G.GEMV_MAX_M and K % 8 == 0
            and K <= 8192 and x.is_contiguous())


def _gemv_prologue(x: NormedRows, w, epi: str, plan: Optional[G.GemmPlan], C, ldc, ws=None):
    """Run the GEMV with the deferred norm in its prologue; False if the plan has no such
    variant (the caller materialises the norm)."""
    M, K = x.shape
    p = plan or G.plan(M, w.shape[0], K, epi)
    tiles = G.GEMV_PRO_TILES.get(epi, ())
    if p.tile not in tiles or (p.tile in G.GEMV_PRO_M1_ONLY and M > 1) or M > G.GEMV_MAX_M:
        return False
    r = x.residual
    code = G.EPI["silu_mul"] if epi == "silu_mul" else 0
    if ws is None and p.splits > 1:      # split K into C: slabs + the reduce kernel
        ws = G.workspace(r.device, p.splits * M * w.shape[0] * 4)
    _native_call("dli_gemv_fused", _p(r), r.stride(0), _p(x.w), x.eps, _p(w), w.stride(-2),
                 _p(C), ldc, M, w.shape[0], K, code, p.tile, p.splits, _p(ws), _st())
    return True


def linear_normed(x: NormedRows, w, epi: str, plan: G.GemmPlan):
    """epi(rmsnorm(x) @ w.T) under a forced plan (the autotuner's timing of a prologue GEMV;
    plans without a prologue variant materialise the norm first, as ``linear`` does)."""
    n_out = w.shape[-2] // 2 if epi == "silu_mul" else w.shape[-2]
    y = torch.empty(x.shape[0], n_out, dtype=x.dtype, device=x.device)
    if plan.splits > 1 and epi == "splitk":
        return _gemm_native(x.materialize(), w, "none", plan=plan)
    if _gemv_prologue(x, w, epi, plan, y, y.stride(0)):
        return y
    return _gemm_native(x.materialize(), w, epi, plan=plan, out=y)


def linear_residual(x, w, residual, plan: Optional[G.GemmPlan] = None):
    """residual += x @ w.T (bf16-rounded, in place) — the O / down projection of a batch-1
    decode layer as ONE kernel: full K per workgroup, the add in its epilogue (no split-K
    slabs, no reduce kernel). Other shapes take ``linear_add_rmsnorm`` without a norm."""
    M, K = x.shape
    p = plan or G.plan(M, w.shape[0], K, "res")
    if (not _use_native(x) or p.tile not in G.GEMV_RES_TILES or M > G.GEMV_MAX_M
            or not residual.is_contiguous() or x.stride(-1) != 1 or w.stride(-1) != 1):
        linear_add_rmsnorm(x, w, residual, None, 0.0)
        return
    _native_call("dli_gemv_fused", _p(x), x.stride(0), None, 0.0, _p(w), w.stride(-2),
                 _p(residual), residual.stride(0), M, w.shape[0], K, 16, p.tile, 1, None, _st())


# ----------------------------------------------------------------------------- embedding
def embedding(ids, table, pos_table=None, positions=None):
    if not _use_native(table):
        return R.embedding(ids, table, pos_table, positions)
    T = ids.shape[0]
    out = torch.empty(T, table.shape[1], dtype=table.dtype, device=table.device)
    _native_call("dli_embedding", _p(out), _p(ids), _p(table), _p(pos_table), _p(positions), T,
                 table.shape[1], _st())
    return out


# ----------------------------------------------------------------------------- GEMM
def _gemm_native(x, w, epi: str, bias=None, out=None, plan: Optional[G.GemmPlan] = None,
                 groups: int = 1, group_off=None, rows_per_group: Optional[int] = None):
    M, K = x.shape
    Nn = w.shape[-2]
    if plan is None:
        if group_off is None:
            plan = G.plan(M, Nn, K, epi)
        else:
            plan = G.grouped_plan(M, Nn, K, epi, groups)
    out_n = Nn // 2 if epi == "silu_mul" else Nn
    if out is None:
        dt = torch.float32 if epi == "f32" else x.dtype
        out = torch.empty(M, out_n, dtype=dt, device=x.device)
    splits = plan.splits
    ws = None
    if splits > 1:
        ws = G.workspace(x.device, splits * M * Nn * 4)
    m_arg = M if group_off is None else rows_per_group
    _native_call("dli_gemm", _p(x), x.stride(0), _p(w), w.stride(-2), _p(out), out.stride(0),
                 m_arg, Nn, K, G.EPI[epi], plan.tile, splits, _p(bias), _p(ws), _p(group_off),
                 groups, _st())
    return out


def linear(x, w, bias=None, epi: str = "none", out=None):
    """y = epi(x @ w.T (+bias)). epi in {none, f32, silu_mul, bias_gelu, bias}.
    silu_mul expects the 16-row interleaved gate/up weight and returns width N/2."""
    if bias is not None and epi == "none":
        epi = "bias"
    if isinstance(x, NormedRows):
        if (bias is None and epi in ("none", "silu_mul") and _use_native(x.residual)
                and x.residual.is_contiguous()):
            M = x.shape[0]
            n_out = w.shape[-2] // 2 if epi == "silu_mul" else w.shape[-2]
            y = out if out is not None else torch.empty(M, n_out, dtype=x.dtype, device=x.device)
            if _gemv_prologue(x, w, epi, None, y, y.stride(0)):
                return y
        x = x.materialize()
    if not _use_native(x):
        if epi == "silu_mul":
            y = R.silu_mul(R.linear(x, w))
        elif epi == "f32":
            y = R.linear(x, w, out_dtype=torch.float32)
        elif epi == "bias_gelu":
            y = R.gelu_tanh(R.linear(x, w, bias))
        else:
            y = R.linear(x, w, bias)
        if out is not None:
            out.copy_(y)
            return out
        return y
    if x.stride(-1) != 1 or w.stride(-1) != 1:
        raise ValueError("linear: inner dims must be contiguous")
    return _gemm_native(x, w, epi, bias=bias, out=out)


def _slab_gemm(x, w, p: G.GemmPlan, ws) -> int:
    """x @ w.T as ``p.splits`` split-K partial slabs in ``ws`` (no output tensor: a fused
    consumer reduces them). Returns the slab format the consumer must read: 1 = fp16 x 1/16
    (the MFMA families' EPI "slab16" store, half the bytes), 0 = fp32."""
    M, K = x.shape
    Nn = w.shape[0]
    fmt = 1 if (G.SLAB16 and p.tile in G.SLAB16_TILES and p.splits in (2, 4, 8)) else 0
    _native_call("dli_gemm", _p(x), x.stride(0), _p(w), w.stride(-2), None, Nn, M, Nn, K,
                 G.EPI["slab16"] if fmt else 0, p.tile, p.splits, None, _p(ws), None, 1, _st())
    return fmt


def _splitk_plan(x, w):
    """A split-K plan for a GEMM whose partial sums feed a fused reduce, or None."""
    if not _use_native(x) or x.stride(-1) != 1 or w.stride(-1) != 1:
        return None
    M, K = x.shape
    p = G.plan(M, w.shape[0], K, "splitk")
    return p if p.splits > 1 else None


def linear_add_rmsnorm(x, w, residual, norm_w, eps, plan: Optional[G.GemmPlan] = None,
                       route=None):
    """residual += x @ w.T (bf16-rounded, in place); returns rmsnorm(residual) * norm_w
    (None when norm_w is None). Split-K GEMMs reduce their partial slabs inside the norm
    kernel (fused_reduce.hip), so the bf16 GEMM output is never materialised.
    ``plan`` forces the GEMM plan (the autotuner times every candidate with its consumer).
    ``route`` = (router weight [E, N], k): also the MoE gate of the output rows — returns
    (out, topk_w, topk_ids); with fp16 slabs, N = 4096 and E <= 8 inside the same reduce
    kernel (``dli_splitk_add_rmsnorm_route``), else by ``moe_router``."""
    if route is not None:
        wr, k = route
        p = _splitk_plan(x, w) if plan is None else (plan if plan.splits > 1 else None)
        M, K = x.shape
        Nn = w.shape[0]
        if (p is not None and norm_w is not None and Nn == 4096 and wr.shape[0] <= 8
                and wr.is_contiguous() and residual.is_contiguous()
                and wr.data_ptr() % 16 == 0):
            ws = G.workspace(x.device, p.splits * M * Nn * 4)
            fmt = _slab_gemm(x, w, p, ws)
            if fmt == 1:
                out = torch.empty_like(residual)
                tw = torch.empty(M, k, dtype=torch.float32, device=x.device)
                ti = torch.empty(M, k, dtype=torch.int32, device=x.device)
                _native_call("dli_splitk_add_rmsnorm_route", _p(out), _p(residual), _p(ws),
                             p.splits, M, Nn, _p(norm_w), eps, _p(wr), wr.shape[0], k, _p(tw),
                             _p(ti), _st())
                return out, tw, ti
            out = torch.empty_like(residual)
            _native_call("dli_splitk_add_rmsnorm", _p(out), _p(residual), _p(ws), p.splits, M,
                         Nn, _p(norm_w), eps, fmt, _st())
        else:
            out = linear_add_rmsnorm(x, w, residual, norm_w, eps, plan=plan)
        return (out,) + tuple(moe_router(out, wr, k))
    if plan is None:
        p = _splitk_plan(x, w)
    else:
        p = plan if plan.splits > 1 else None
    if p is None:
        y = linear(x, w) if plan is None else _gemm_native(x, w, "none", plan=plan)
        if norm_w is None:
            residual.add_(y)             # bf16 add computes in fp32 and rounds once
            return None
        return add_rmsnorm(y, residual, norm_w, eps)
    M, K = x.shape
    Nn = w.shape[0]
    ws = G.workspace(x.device, p.splits * M * Nn * 4)
    out = torch.empty_like(residual) if norm_w is not None else None
    fmt = _slab_gemm(x, w, p, ws)
    _native_call("dli_splitk_add_rmsnorm", _p(out), _p(residual), _p(ws), p.splits, M, Nn,
                 _p(norm_w), eps, fmt, _st())
    return out


def linear_rope_cache(x, w, positions, slot_mapping, cos_sin, k_cache, v_cache, hq, hkv, hd,
                      use_rope: bool = True, plan: Optional[G.GemmPlan] = None):
    """qkv = x @ w.T with RoPE applied in place to q,k and k,v written to the paged cache.
    ``plan`` forces the GEMM plan (the autotuner times QKV candidates with this consumer)."""
    if isinstance(x, NormedRows):
        x = x.materialize()
    if plan is None:
        p = _splitk_plan(x, w)
    else:
        p = plan if plan.splits > 1 else None
    if p is None:
        qkv = linear(x, w) if plan is None else _gemm_native(x, w, "none", plan=plan)
        rope_and_cache(qkv, positions, slot_mapping, cos_sin, k_cache, v_cache, hq, hkv, hd,
                       use_rope)
        return qkv
    M, K = x.shape
    Nn = w.shape[0]
    ws = G.workspace(x.device, p.splits * M * Nn * 4)
    fmt = _slab_gemm(x, w, p, ws)
    qkv = torch.empty(M, Nn, dtype=x.dtype, device=x.device)
    bs = k_cache.shape[2] if k_cache is not None else 16
    _native_call("dli_splitk_rope_cache", _p(qkv), _p(ws), p.splits, M, Nn, _p(positions),
                 _p(slot_mapping), _p(cos_sin), _p(k_cache), _p(v_cache), hq, hkv, hd, bs,
                 int(use_rope), fmt, _st())
    return qkv


def linear_rope_attention(x, w, positions, slot_mapping, cos_sin, k_cache, v_cache,
                          block_tables, context_lens, max_context: int, hq, hkv, hd, scale):
    """Decode step, one fused pass after the QKV GEMM: the split-K slabs (or, for an unsplit
    plan, the bf16 QKV rows) are reduced, q and k rotated, k/v written to the paged cache and
    attention computed by ONE kernel per layer (``dli_decode_attention_fused``) instead of
    ``linear_rope_cache`` + ``decode_attention``. Returns the attention output [B, hq*hd], or
    None where the fused kernel does not apply (the caller then runs the two-kernel path):
    split counts other than 2 / 4, KV-split attention (long contexts at small batch), the
    pipelined long-context kernel, head dim != 128."""
    xr = x.residual if isinstance(x, NormedRows) else x
    if hd != 128 or k_cache is None or not _use_native(xr):
        return None
    p = _splitk_plan(xr, w)
    if p is not None and p.splits not in (2, 4):
        return None
    B, K = x.shape
    if decode_num_splits(B, hkv, max_context) != 1:
        return None
    mode = int(N.require_native().dli_decode_get_pipe())
    if mode == 1 or (mode == 2 and -(-max_context // 32) * 32 >= 768):
        return None                       # dli_decode_attention picks the pipelined kernel
    Nn = w.shape[0]
    fmt = 0
    if p is None:                         # unsplit plan: the prologue reads the bf16 rows
        src, splits = linear(x, w), 0
    else:
        src, splits = G.workspace(xr.device, p.splits * B * Nn * 4), p.splits
        if not (isinstance(x, NormedRows)
                and _gemv_prologue(x, w, "splitk", p, None, Nn, ws=src)):
            if isinstance(x, NormedRows):
                x = x.materialize()
            fmt = _slab_gemm(x, w, p, src)
    out = torch.empty(B, hq * hd, dtype=x.dtype, device=x.device)
    _native_call("dli_decode_attention_fused", _p(out), _p(src), splits, _p(positions),
                 _p(slot_mapping), _p(cos_sin), _p(k_cache), _p(v_cache), _p(block_tables),
                 block_tables.stride(0), _p(context_lens), B, hq, hkv, hd, k_cache.shape[2],
                 scale, fmt, _st())
    return out


def feed_ids(ids, src, feed):
    """In place: ids[i] = feed[src[i]] where src[i] >= 0 (int32 tensors; lookahead input ids
    taken from the in-flight step's sampled tokens)."""
    if not _use_native(ids):
        take = feed.index_select(0, src.clamp(min=0).long()).to(ids.dtype)
        ids.copy_(torch.where(src >= 0, take, ids))
        return ids
    if ids.dtype != torch.int32 or src.dtype != torch.int32 or feed.dtype != torch.int32:
        raise ValueError("feed_ids: int32 tensors expected")
    _native_call("dli_feed_ids", _p(ids), _p(src), _p(feed), ids.shape[0], feed.shape[0], _st())
    return ids


_sinks: dict = {}


def prefetch(t: torch.Tensor, max_wgs: int = 256, nbytes: Optional[int] = None) -> None:
    """Read ``t`` (its first ``nbytes``) on the current stream and discard it: the weight
    lands in the Infinity Cache for the GEMM that streams it next (see
    ``TransformerLM._llama_layers``). No-op off the GPU."""
    if not _use_native(t):
        return
    sink = _sinks.get(t.device)
    if sink is None:
        sink = _sinks[t.device] = torch.empty(256, dtype=torch.int32, device=t.device)
    n = t.numel() * t.element_size() if nbytes is None else int(nbytes)
    _native_call("dli_prefetch", _p(t), n, int(max_wgs), _p(sink), _st())


def silu_mul(gu):
    if not _use_native(gu):
        return R.silu_mul(gu)
    T, F2 = gu.shape
    out = torch.empty(T, F2 // 2, dtype=gu.dtype, device=gu.device)
    _native_call("dli_silu_mul", _p(out), _p(gu), T, F2 // 2, _st())
    return out


def bias_act_(x, bias, act: str = "none"):
    if not _use_native(x):
        y = x.float() + (bias.float() if bias is not None else 0)
        if act == "gelu":
            y = torch.nn.functional.gelu(y, approximate="tanh")
        x.copy_(y.to(x.dtype))
        return x
    T, Nn = x.shape
    _native_call("dli_bias_act", _p(x), _p(bias), T, Nn, 1 if act == "gelu" else 0, _st())
    return x


# ----------------------------------------------------------------------------- RoPE / KV cache
def rope_and_cache(qkv, positions, slot_mapping, cos_sin, k_cache, v_cache, hq, hkv, hd,
                   use_rope: bool = True):
    """In-place RoPE on q,k inside qkv + paged cache write. Returns views (q, k, v)."""
    if not _use_native(qkv):
        return R.rope_and_cache(qkv, positions, slot_mapping, cos_sin, k_cache, v_cache, hq, hkv,
                                hd, use_rope)
    T = qkv.shape[0]
    bs = k_cache.shape[2] if k_cache is not None else 16
    _native_call("dli_rope_cache", _p(qkv), qkv.stride(0), _p(positions), _p(slot_mapping),
                 _p(cos_sin), _p(k_cache), _p(v_cache), T, hq, hkv, hd, bs, int(use_rope), _st())
    return R.split_qkv(qkv, hq, hkv, hd)


# ----------------------------------------------------------------------------- attention
def prefill_attention(qkv, cu_seqlens, max_seqlen: int, hq, hkv, hd, scale, out=None):
    """Causal varlen attention over the packed prompt tokens in ``qkv``; returns [T, Hq*hd]."""
    T = qkv.shape[0]
    if not _use_native(qkv):
        q, k, v = R.split_qkv(qkv, hq, hkv, hd)
        o = R.prefill_attention(q, k, v, cu_seqlens, scale).reshape(T, hq * hd)
        if out is not None:
            out.copy_(o)
            return out
        return o
    if out is None:
        out = torch.empty(T, hq * hd, dtype=qkv.dtype, device=qkv.device)
    nseq = cu_seqlens.shape[0] - 1
    _native_call("dli_prefill_attention", _p(out), out.stride(0), _p(qkv), qkv.stride(0),
                 _p(cu_seqlens), nseq, max_seqlen, hq, hkv, hd, scale, _st())
    return out


def decode_pipelined(v: int) -> int:
    """Select the pipelined (1), one-tile-per-round (0) or automatic (2, the default: pipelined
    for KV splits of >= 768 tokens) decode attention kernel for head_dim 128. Returns the
    previous setting (tests force either kernel with it)."""
    return int(N.require_native().dli_decode_set_pipe(int(v)))


def decode_form(v: int) -> int:
    """Force the unsplit decode attention's form: 1 = a wave per (sequence, kv head), 4 = a
    workgroup per item, 0 = automatic (workgroup per item for <= 256 items). Returns the
    previous setting (tests force either form with it)."""
    return int(N.require_native().dli_decode_set_form(int(v)))


def prefill_long_min_len(n: int = 0) -> int:
    """Shortest max_seqlen routed to the 256-row (32x32x16) prefill attention kernel; n > 0
    sets it. Returns the previous value (A/B runs and tests force either kernel with it)."""
    return int(N.require_native().dli_prefill_set_min_len(int(n)))


def prefill_set_pack(on: bool) -> bool:
    """Head packing of the short-prompt prefill attention kernel (2 / 4 query heads of a GQA
    group per workgroup when every prompt of the batch is <= 32 / 16 tokens); returns the
    previous setting (A/B switch, on by default)."""
    return bool(N.require_native().dli_prefill_set_pack(1 if on else 0))


def prefill_attention_paged(qkv, cu_seqlens, max_seqlen: int, context_lens, block_tables,
                            k_cache, v_cache, hq, hkv, hd, scale, out=None):
    """Chunked prefill attention: each sequence's chunk of queries (packed rows of ``qkv``)
    attends over all ``context_lens[i]`` keys of the sequence in the paged cache — earlier
    chunks plus this one (already written by ``rope_and_cache``); [T, Hq*hd]."""
    T = qkv.shape[0]
    if not _use_native(qkv):
        q = qkv[:, : hq * hd].reshape(T, hq, hd)
        o = R.prefill_attention_paged(q, k_cache, v_cache, cu_seqlens, context_lens,
                                      block_tables, scale).reshape(T, hq * hd)
        if out is not None:
            out.copy_(o)
            return out
        return o
    if out is None:
        out = torch.empty(T, hq * hd, dtype=qkv.dtype, device=qkv.device)
    nseq = cu_seqlens.shape[0] - 1
    _native_call("dli_prefill_attention_paged", _p(out), out.stride(0), _p(qkv), qkv.stride(0),
                 _p(cu_seqlens), _p(context_lens), _p(k_cache), _p(v_cache), _p(block_tables),
                 block_tables.stride(0), nseq, max_seqlen, hq, hkv, hd, k_cache.shape[2], scale,
                 _st())
    return out


def decode_num_splits(B: int, hkv: int, max_context: int) -> int:
    """KV splits so that the B*Hkv*splits work items (one wave each) fill the chip's ~2048
    resident waves for long contexts, keeping >= 128 tokens per split."""
    items = B * hkv
    splits = 1
    # tiny batches (batch-1 latency): >= 512 tokens per split, so graphs captured for a
    # 512-token table take the single-pass kernel with the fused QKV reduce / RoPE / cache
    # prologue (the 4-split form cost rope + attention + merge = 23 us per layer at B = 1,
    # profiles/r3/prof_b1_summary.txt)
    min_tok = 512 if B <= 4 else 128
    while items * splits < 2048 and max_context // (splits * 2) >= min_tok and splits < 64:
        splits *= 2
    return splits


def decode_attention(qkv, k_cache, v_cache, block_tables, context_lens, max_context: int,
                     hq, hkv, hd, scale, out=None, num_splits: Optional[int] = None):
    """One query per row of ``qkv`` (rows = sequences) against its paged KV; [B, Hq*hd]."""
    B = qkv.shape[0]
    if not _use_native(qkv):
        q = qkv[:, : hq * hd].reshape(B, hq, hd)
        o = R.decode_attention(q, k_cache, v_cache, block_tables, context_lens,
                               scale).reshape(B, hq * hd)
        if out is not None:
            out.copy_(o)
            return out
        return o
    if out is None:
        out = torch.empty(B, hq * hd, dtype=qkv.dtype, device=qkv.device)
    if num_splits is None:
        num_splits = decode_num_splits(B, hkv, max_context)
    ws = None
    if num_splits > 1:
        nbytes = B * hq * num_splits * (hd + 2) * 4
        ws = G.workspace(qkv.device, nbytes)
    bs = k_cache.shape[2]
    _native_call("dli_decode_attention", _p(out), _p(qkv), qkv.stride(0), _p(k_cache),
                 _p(v_cache), _p(block_tables), block_tables.stride(0), _p(context_lens), B, hq,
                 hkv, hd, bs, scale, max_context, num_splits, _p(ws), _st())
    return out


# ----------------------------------------------------------------------------- sampling
_sample_wss: dict = {}


def _sample_ws(device, B: int, V: int):
    """Zero-initialised scratch of the two-phase small-batch sampler (sampling.hip
    sample_chunk_kernel: B <= 8 rows split over up to 64 workgroups each), or None. One buffer
    per device, sized for the largest batch; the kernels leave its overflow flags zero."""
    lib = N.require_native()
    if int(lib.dli_sample_workspace_bytes(B, V)) == 0:
        return None
    key = (device.type, device.index)
    ws = _sample_wss.get(key)
    nbytes = int(lib.dli_sample_workspace_bytes(B, V))
    if ws is None or ws.numel() < nbytes:
        # sized for the largest two-phase batch (the library's split limit; 8 by default)
        maxb = int(lib.dli_sample_set_split_max_b(0))
        nbytes = max(nbytes, int(lib.dli_sample_workspace_bytes(maxb, V)))
        if ws is not None:
            G._retired.append(ws)        # a captured graph may still hold it (ops.gemm)
        ws = _sample_wss[key] = torch.zeros(nbytes, dtype=torch.uint8, device=device)
    return ws


# LM-head output dtype: fp32 (the head GEMM accumulates in fp32 and stores it). bf16 logits
# were measured without a gain at batch 512 (profiles/r5/s05/ab.jsonl: the head GEMM is
# MFMA-bound at the same 407 us either way) and make a request's draws depend on which GEMM
# plan (batch size) rounded its logits, which breaks batch-invariant seeded sampling.
HEAD_EPI = "f32"


def sample(logits, temperature, top_k, top_p, seeds, generator=None, ids=None):
    """logits fp32 or bf16 [B, V] -> int32 tokens [B] (every comparison on the exact fp32
    value of each logit). temperature<=0 -> greedy. With ``ids``
    [B, V] the row holds candidates (vocab-parallel LM head) in ascending token-id order,
    and the sampled column is mapped to its token id (ties then break by token id exactly
    as over the full vocabulary)."""
    if not _use_native(logits):
        return R.sample(logits, temperature, top_k, top_p, generator=generator, seeds=seeds,
                        ids=ids)
    B, V = logits.shape
    out = torch.empty(B, dtype=torch.int32, device=logits.device)
    if logits.dtype not in (torch.float32, torch.bfloat16):
        logits = logits.float()
    fn = "dli_sample_bf16" if logits.dtype == torch.bfloat16 else "dli_sample"
    _native_call(fn, _p(out), _p(logits), logits.stride(0), B, V, _p(temperature),
                 _p(top_k), _p(top_p), _p(seeds), _p(_sample_ws(logits.device, B, V)), _st())
    if ids is not None:
        out = ids.gather(1, out.long().unsqueeze(1)).squeeze(1).to(torch.int32)
    return out


def head_candidates(h, w_slice, offset: int, c: int):
    """Vocab-parallel LM head slice on this rank: logits (``HEAD_EPI``: the model dtype, as
    the single-stage head) for token ids ``[offset, offset + V_r)`` and the top-``c`` per
    row (ties broken by the lower token id), returned in ascending token-id order (values
    fp32 [S, c], ids int32 [S, c]). The union over ranks contains every token a top-k <= c
    sampler can pick."""
    lg = linear(h, w_slice, epi=HEAD_EPI)
    S, V = lg.shape
    c = min(c, V)
    if not _use_native(h):
        # stable descending sort: equal logits keep ascending token-id order
        v, i = torch.sort(lg.float(), dim=-1, descending=True, stable=True)
        v, i = v[:, :c], (i[:, :c] + offset).to(torch.int32)
        i, perm = torch.sort(i, dim=-1)
        return v.gather(1, perm), i
    v = torch.empty(S, c, dtype=torch.float32, device=h.device)
    i = torch.empty(S, c, dtype=torch.int32, device=h.device)
    # HIP top-c per row, written in ascending id order (sampling.hip topk_rows_kernel)
    fn = "dli_topk_rows_bf16" if lg.dtype == torch.bfloat16 else "dli_topk_rows"
    _native_call(fn, _p(v), _p(i), _p(lg), lg.stride(0), S, V, c, int(offset), _st())
    return v, i


# ----------------------------------------------------------------------------- MoE
def moe_route(router_logits, k: int):
    if not _use_native(router_logits):
        return R.router_topk(router_logits, k)
    T, E = router_logits.shape
    w = torch.empty(T, k, dtype=torch.float32, device=router_logits.device)
    ids = torch.empty(T, k, dtype=torch.int32, device=router_logits.device)
    _native_call("dli_moe_route", _p(w), _p(ids), _p(router_logits), T, E, k, _st())
    return w, ids


def moe_router(h, w_router, k: int):
    """The MoE gate: logits = h @ w_router.T (bf16, as a GEMM would write them), softmax,
    top-``k``, renormalised. On the GPU with <= 8 experts one kernel does all of it
    (``moe_router_kernel``, a wave per token); else the GEMM then ``moe_route``."""
    T, D = h.shape
    E = w_router.shape[0]
    if (_use_native(h) and E <= 8 and D % 8 == 0 and h.stride(-1) == 1
            and h.stride(0) % 8 == 0 and w_router.is_contiguous()
            and h.data_ptr() % 16 == 0 and w_router.data_ptr() % 16 == 0):
        w = torch.empty(T, k, dtype=torch.float32, device=h.device)
        ids = torch.empty(T, k, dtype=torch.int32, device=h.device)
        _native_call("dli_moe_router", _p(w), _p(ids), _p(h), h.stride(0), _p(w_router), T, E,
                     D, k, _st())
        return w, ids
    return moe_route(linear(h, w_router), k)


def moe_mlp(x, w_gu, w_down, topk_w, topk_ids, expert_offset: int = 0,
            plan_rows: Optional[int] = None, defer_combine: bool = False):
    """Experts [expert_offset, expert_offset+E_local) of one MoE layer; returns the weighted
    sum over the token's selected local experts (zeros for tokens routed elsewhere).
    ``plan_rows``: the routed rows these experts typically receive, when ``x`` is a region
    sized for the worst case (the expert-parallel receive region: every peer's bucket at
    min(k, E/N) rows per token). The grouped-GEMM plan is looked up for it — the autotuned
    key — instead of for the capacity, whose 4-8x larger row count mapped to 256-row tiles
    (1 workgroup per CU) that streamed the experts at ~2 TB/s."""
    if not _use_native(x):
        return R.moe_mlp(x, w_gu, w_down, topk_w, topk_ids, expert_offset)
    T, D = x.shape
    k = topk_ids.shape[1]
    E_local, F2, _ = w_gu.shape
    n = T * k
    dev = x.device
    offsets = torch.empty(E_local + 1, dtype=torch.int32, device=dev)
    pos = torch.empty(n, dtype=torch.int32, device=dev)
    src = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
    _native_call("dli_moe_align", _p(offsets), _p(pos), _p(src), _p(topk_ids), n, k,
                 expert_offset, E_local, _st())
    act = torch.empty(max(n, 1), F2 // 2, dtype=x.dtype, device=dev)
    if n >= _MOE_PREFILL_ROWS * E_local and not torch.cuda.is_current_stream_capturing():
        # prefill-sized expert GEMMs (thousands of rows per expert) are compute-bound: a
        # grouped 256x256 kernel (G.MOE_PREFILL_TILE: the two-barrier 4-wave tile, grid.z =
        # expert) with the fused SiLU*up epilogue. The largest expert's row count bounds the
        # grid (one host read of the offsets per MoE layer, eager prefill only) instead of n,
        # which would launch ~8x more (empty) row tiles per expert.
        xp = torch.empty(max(n, 1), D, dtype=x.dtype, device=dev)
        _native_call("dli_moe_gather", _p(xp), _p(x), _p(src), n, D, _p(offsets[E_local:]),
                     _st())
        offs = offsets.tolist()
        rows_max = max(b - a for a, b in zip(offs[:-1], offs[1:]))
        y = torch.empty(max(n, 1), D, dtype=x.dtype, device=dev)
        if rows_max > 0:
            p8 = G.GemmPlan("dli", G.MOE_PREFILL_TILE, 1)
            _gemm_native(xp, w_gu, "silu_mul", out=act, groups=E_local, group_off=offsets,
                         rows_per_group=rows_max, plan=p8)
            _gemm_native(act, w_down, "none", out=y, groups=E_local, group_off=offsets,
                         rows_per_group=rows_max, plan=p8)
        out = torch.empty_like(x)
        _native_call("dli_moe_combine", _p(out), _p(y), _p(topk_w), _p(pos), T, k, D, _st())
        return out
    rows = plan_rows if plan_rows is not None else n
    p_gu = G.grouped_plan(rows, F2, D, "silu_mul", E_local)
    if p_gu.splits == 1 and p_gu.tile in G.GATHER_TILES and x.is_contiguous():
        # the gate/up GEMM reads the token rows in place through the permutation (no gathered
        # copy of them: dli_gemm_grouped_gather, the generic tile family)
        _native_call("dli_gemm_grouped_gather", _p(x), x.stride(0), _p(w_gu), w_gu.stride(-2),
                     _p(act), act.stride(0), n, F2, D, p_gu.tile, _p(src), _p(offsets),
                     E_local, _st())
    else:
        # permuted rows: at most n (all local); rows past offsets[E_local] are never touched
        xp = torch.empty(max(n, 1), D, dtype=x.dtype, device=dev)
        _native_call("dli_moe_gather", _p(xp), _p(x), _p(src), n, D, _p(offsets[E_local:]),
                     _st())
        _gemm_native(xp, w_gu, "silu_mul", out=act, groups=E_local, group_off=offsets,
                     rows_per_group=n, plan=p_gu)
    p_dn = G.grouped_plan(rows, D, F2 // 2, "none", E_local)
    if moe_slab_plan(p_dn):
        if defer_combine:
            # the down projection's slabs; the combine runs with the next layer's add + norm
            ws = G.workspace(dev, p_dn.splits * max(n, 1) * D * 2)
            _native_call("dli_gemm", _p(act), act.stride(0), _p(w_down), w_down.stride(-2),
                         None, D, n, D, F2 // 2, G.EPI["slab16"], p_dn.tile, p_dn.splits, None,
                         _p(ws), _p(offsets), E_local, _st())
            return MoEPending(ws, p_dn.splits, n, topk_w, pos, (T, D), x.dtype, dev)
        out = torch.empty_like(x)
        moe_down_combine(act, w_down, offsets, n, p_dn, topk_w, pos, out)
        return out
    y = torch.empty(max(n, 1), D, dtype=x.dtype, device=dev)
    _gemm_native(act, w_down, "none", out=y, groups=E_local, group_off=offsets,
                 rows_per_group=n, plan=p_dn)
    out = torch.empty_like(x)
    _native_call("dli_moe_combine", _p(out), _p(y), _p(topk_w), _p(pos), T, k, D, _st())
    return out


def moe_slab_plan(p: Optional[G.GemmPlan]) -> bool:
    """Whether a grouped down-projection plan runs as fp16 split-K slabs reduced inside the
    combine (``moe_down_combine``) instead of GEMM -> fp32 slab reduce -> bf16 y -> combine."""
    return (p is not None and G.SLAB16 and p.splits in (2, 4, 8)
            and p.tile in G.SLAB16_TILES)


def moe_down_combine(act, w_down, offsets, n: int, p: G.GemmPlan, topk_w, pos, out):
    """Grouped down projection of the ``n`` permuted rows ``act`` as fp16 split-K slabs
    (EPI "slab16"), reduced by the combine itself: out[t] = sum_j topk_w[t, j] *
    bf16(sum_s slab_s[pos[t * k + j]]) (csrc/kernels/moe.hip moe_combine_slabs_kernel)."""
    E_local, D, F = w_down.shape
    ws = G.workspace(act.device, p.splits * max(n, 1) * D * 2)
    _native_call("dli_gemm", _p(act), act.stride(0), _p(w_down), w_down.stride(-2), None, D,
                 n, D, F, G.EPI["slab16"], p.tile, p.splits, None, _p(ws), _p(offsets),
                 E_local, _st())
    T, k = topk_w.shape                  # pos: [T * k] rows (flat, as moe_align writes it)
    _native_call("dli_moe_combine_slabs", _p(out), _p(ws), p.splits, n, _p(topk_w), _p(pos),
                 T, k, D, _st())
    return out


def ep_pack(x, topk_ids, e_per: int, base, send_rows: int, counts: bool = False):
    """Expert-parallel dispatch: (token, pick) rows into per-destination-rank buckets
    starting at ``base[dest]`` (int32 [N] on the device). Returns (send_x [send_rows, D],
    send_e int32 [send_rows] global expert id or -1, pos int32 [T, k] row of each pick)
    and, with ``counts``, the rows per destination (int32 [N] on the device)."""
    T, D = x.shape
    k = topk_ids.shape[1]
    dev = x.device
    send_x = torch.empty(max(send_rows, 1), D, dtype=x.dtype, device=dev)[:send_rows]
    send_e = torch.full((send_rows,), -1, dtype=torch.int32, device=dev)
    pos = torch.empty(T, k, dtype=torch.int32, device=dev)
    if not _use_native(x):
        # deterministic reference: slots in (token, pick) order
        fill = [0] * base.shape[0]
        bl = base.tolist()
        ids = topk_ids.tolist()
        for t in range(T):
            for j in range(k):
                d = ids[t][j] // e_per
                p = bl[d] + fill[d]
                fill[d] += 1
                pos[t, j] = p
                send_e[p] = ids[t][j]
                send_x[p] = x[t]
        if counts:
            return send_x, send_e, pos, torch.tensor(fill, dtype=torch.int32)
        return send_x, send_e, pos
    fill = torch.zeros(base.shape[0], dtype=torch.int32, device=dev)
    if T > 0:
        _native_call("dli_ep_pack", _p(send_x), _p(send_e), _p(pos), _p(fill), _p(base), _p(x),
                     _p(topk_ids), T, k, D, e_per, _st())
    if counts:
        return send_x, send_e, pos, fill
    return send_x, send_e, pos


def moe_combine(y, topk_w, pos):
    """out[t] = sum_j topk_w[t, j] * y[pos[t, j]] (fp32 sum in j order, bf16 out); pos < 0
    rows contribute nothing."""
    T, k = pos.shape
    D = y.shape[1]
    if not _use_native(y):
        out = torch.zeros(T, D, dtype=torch.float32, device=y.device)
        for j in range(k):
            pj = pos[:, j].long()
            ok = pj >= 0
            out[ok] += topk_w[ok, j:j + 1].float() * y[pj[ok]].float()
        return out.to(y.dtype)
    out = torch.empty(T, D, dtype=y.dtype, device=y.device)
    _native_call("dli_moe_combine", _p(out), _p(y), _p(topk_w), _p(pos), T, k, D, _st())
    return out


# ----------------------------------------------------------------------------- misc
def native_library_path():
    return N.loaded_path()


def benchmark(fn, iters: int = 20, warmup: int = 3, graph: bool = False) -> float:
    """Median milliseconds of fn() on the current stream (GPU) or wall clock (CPU).
    ``graph=True`` captures fn() in a HIP graph and times replays: the GPU time of a
    launch-bound sequence as a decode graph runs it. Timed eagerly, a batch-1 GEMM (~15 us)
    plus its consumer kernel cost less GPU time than the host spends launching them, so the
    autotuner compared host launch overheads and picked plans at random (two runs of the
    same bench took different decode paths)."""
    for _ in range(warmup):
        fn()
    if graph and torch.cuda.is_available():
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            with torch.cuda.graph(g, stream=side):
                fn()
        torch.cuda.current_stream().wait_stream(side)
        g.replay()
        torch.cuda.synchronize()
        times = []
        for _ in range(iters):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            g.replay()
            e.record()
            e.synchronize()
            times.append(s.elapsed_time(e))
        del g
        times.sort()
        return times[len(times) // 2]
    if torch.cuda.is_available():
        torch.cuda.synchronize()
        times = []
        for _ in range(iters):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            fn()
            e.record()
            e.synchronize()
            times.append(s.elapsed_time(e))
    else:
        times = []
        for _ in range(iters):
            t0 = time.perf_counter()
            fn()
            times.append((time.perf_counter() - t0) * 1e3)
    times.sort()
    return times[len(times) // 2]
