"""Pure-PyTorch reference implementations of every hot op (fp32 math).

These are (a) the CPU execution path (config 1: gpt2 on a CPU worker, and every
CPU test), and (b) the golden each HIP kernel is tested against
(SURVEY.md §4 tier T3). They define the tensor layouts the HIP kernels share:

* hidden states: ``[T, D]`` (tokens of all sequences flattened, bf16)
* fused QKV activations: ``[T, (Hq + 2*Hkv) * hd]``
* paged KV cache, per layer:
    ``k_cache [num_blocks, Hkv, block_size, hd]``
    ``v_cache [num_blocks, Hkv, block_size, hd]``  (token-major like K: a decode step's
    K/V write is one contiguous 2*hd-byte row per head; the decode kernel transposes V
    tiles through LDS with ds_read_b64_tr_b16 for its P·V MFMA)
* ``slot_mapping[t] = block * block_size + offset`` (int32)
* gate/up weights interleaved in 16-row groups: rows ``[32i, 32i+16)`` are gate
  features ``[16i, 16i+16)`` and rows ``[32i+16, 32i+32)`` the matching up
  features, so a GEMM tile owns both halves of every SiLU·mul pair.

The implicit HF ops these replace are listed in SURVEY.md §2.4 (K1-K16).
"""
from __future__ import annotations

import math
from typing import Optional, Tuple

import torch
import torch.nn.functional as F

GU_GROUP = 16  # gate/up interleave granularity (rows)


# ----------------------------------------------------------------------------- norms (K2, K3)
def rmsnorm(x: torch.Tensor, w: torch.Tensor, eps: float) -> torch.Tensor:
    xf = x.float()
    var = xf.pow(2).mean(-1, keepdim=True)
    return (xf * torch.rsqrt(var + eps) * w.float()).to(x.dtype)


def fused_add_rmsnorm(x: torch.Tensor, residual: Optional[torch.Tensor], w: torch.Tensor,
                      eps: float) -> Tuple[torch.Tensor, torch.Tensor]:
    """residual' = residual + x (or x when residual is None); out = rmsnorm(residual')."""
    r = x.float() if residual is None else residual.float() + x.float()
    r_out = r.to(x.dtype)
    r = r_out.float()  # the residual stream is bf16 (HF semantics): normalise what is stored
    var = r.pow(2).mean(-1, keepdim=True)
    out = (r * torch.rsqrt(var + eps) * w.float()).to(x.dtype)
    return out, r_out


def layernorm(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor, eps: float) -> torch.Tensor:
    return F.layer_norm(x.float(), (x.shape[-1],), w.float(), b.float(), eps).to(x.dtype)


def fused_add_layernorm(x, residual, w, b, eps):
    r = x.float() if residual is None else residual.float() + x.float()
    r_out = r.to(x.dtype)
    out = F.layer_norm(r_out.float(), (x.shape[-1],), w.float(), b.float(), eps).to(x.dtype)
    return out, r_out


# ----------------------------------------------------------------------------- embedding (K1)
def embedding(ids: torch.Tensor, table: torch.Tensor,
              pos_table: Optional[torch.Tensor] = None,
              positions: Optional[torch.Tensor] = None) -> torch.Tensor:
    x = table[ids.long()]
    if pos_table is not None:
        x = (x.float() + pos_table[positions.long()].float()).to(table.dtype)
    return x


# ----------------------------------------------------------------------------- GEMMs (K4, K9-K12)
def linear(x: torch.Tensor, w: torch.Tensor, bias: Optional[torch.Tensor] = None,
           out_dtype: Optional[torch.dtype] = None) -> torch.Tensor:
    """y = x @ w.T (+ bias); w is [N, K] like torch.nn.Linear."""
    y = x.float() @ w.float().t()
    if bias is not None:
        y = y + bias.float()
    return y.to(out_dtype or x.dtype)


def interleave_gate_up(gate: torch.Tensor, up: torch.Tensor) -> torch.Tensor:
    """[F, K] x2 -> [2F, K] in the 16-row interleaved layout (see module doc)."""
    f, k = gate.shape
    assert f % GU_GROUP == 0, "intermediate size must be a multiple of 16"
    g = gate.reshape(f // GU_GROUP, 1, GU_GROUP, k)
    u = up.reshape(f // GU_GROUP, 1, GU_GROUP, k)
    return torch.cat([g, u], dim=1).reshape(2 * f, k)


def split_gate_up(gu: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """Inverse of the interleave on the last dim of activations [T, 2F]."""
    t, f2 = gu.shape
    v = gu.reshape(t, f2 // (2 * GU_GROUP), 2, GU_GROUP)
    return v[:, :, 0, :].reshape(t, f2 // 2), v[:, :, 1, :].reshape(t, f2 // 2)


def silu_mul(gu: torch.Tensor) -> torch.Tensor:
    g, u = split_gate_up(gu)
    return (F.silu(g.float()) * u.float()).to(gu.dtype)


def gelu_tanh(x: torch.Tensor) -> torch.Tensor:
    return F.gelu(x.float(), approximate="tanh").to(x.dtype)


def linear_silu_mul(x, w_gu):
    return silu_mul(linear(x, w_gu))


# ----------------------------------------------------------------------------- RoPE + KV write (K5, K6)
def rope_cos_sin(max_pos: int, head_dim: int, theta: float, device=None,
                 scaling=()) -> torch.Tensor:
    """[max_pos, head_dim] fp32 table: cols [0, hd/2) = cos, [hd/2, hd) = sin. ``scaling``:
    the HF ``rope_scaling`` of the checkpoint as (key, value) pairs (ModelConfig)."""
    half = head_dim // 2
    inv = 1.0 / (theta ** (torch.arange(0, half, dtype=torch.float64) * 2.0 / head_dim))
    inv = rope_scaled_inv_freq(inv, dict(scaling))
    ang = torch.arange(max_pos, dtype=torch.float64)[:, None] * inv[None, :]
    return torch.cat([ang.cos(), ang.sin()], dim=1).float().to(device)


def rope_scaled_inv_freq(inv: torch.Tensor, sc: dict) -> torch.Tensor:
    """HF ``rope_scaling`` applied to the inverse frequencies (the table absorbs it, so the
    kernels are unchanged). ``llama3``: wavelengths longer than original_max / low_freq_factor
    are divided by ``factor``, shorter than original_max / high_freq_factor kept, the band
    between interpolated (transformers ``_compute_llama3_parameters``); ``linear``: every
    frequency divided by ``factor`` (= positions / factor). Other types are refused."""
    kind = sc.get("rope_type", sc.get("type", "default")) if sc else "default"
    if kind in ("default", None):
        return inv
    factor = float(sc["factor"])
    if kind == "linear":
        return inv / factor
    if kind == "llama3":
        lo, hi = float(sc.get("low_freq_factor", 1.0)), float(sc.get("high_freq_factor", 4.0))
        old = float(sc.get("original_max_position_embeddings", 8192))
        lo_wl, hi_wl = old / lo, old / hi
        wl = 2 * math.pi / inv
        out = torch.where(wl > lo_wl, inv / factor, inv)
        smooth = (old / wl - lo) / (hi - lo)
        smoothed = (1 - smooth) * out / factor + smooth * out
        medium = (wl >= hi_wl) & (wl <= lo_wl)
        return torch.where(medium, smoothed, out)
    raise ValueError(f"unsupported rope_scaling type {kind!r} (supported: llama3, linear)")


def apply_rope(x: torch.Tensor, positions: torch.Tensor, cos_sin: torch.Tensor) -> torch.Tensor:
    """x [T, H, hd] rotate-half RoPE (HF Llama convention), fp32 math."""
    hd = x.shape[-1]
    half = hd // 2
    cs = cos_sin[positions.long()]              # [T, hd]
    cos, sin = cs[:, None, :half], cs[:, None, half:]
    xf = x.float()
    x1, x2 = xf[..., :half], xf[..., half:]
    return torch.cat([x1 * cos - x2 * sin, x2 * cos + x1 * sin], dim=-1).to(x.dtype)


def split_qkv(qkv: torch.Tensor, hq: int, hkv: int, hd: int):
    t = qkv.shape[0]
    q = qkv[:, : hq * hd].reshape(t, hq, hd)
    k = qkv[:, hq * hd: (hq + hkv) * hd].reshape(t, hkv, hd)
    v = qkv[:, (hq + hkv) * hd:].reshape(t, hkv, hd)
    return q, k, v


def write_kv(k: torch.Tensor, v: torch.Tensor, slot_mapping: torch.Tensor,
             k_cache: torch.Tensor, v_cache: torch.Tensor) -> None:
    bs = k_cache.shape[2]
    slots = slot_mapping.long()
    valid = slots >= 0
    slots, kk, vv = slots[valid], k[valid], v[valid]
    blk, off = slots // bs, slots % bs
    k_cache[blk, :, off, :] = kk.to(k_cache.dtype)
    v_cache[blk, :, off, :] = vv.to(v_cache.dtype)


def rope_and_cache(qkv, positions, slot_mapping, cos_sin, k_cache, v_cache,
                   hq: int, hkv: int, hd: int, use_rope: bool = True):
    """Rotates q and k IN PLACE inside ``qkv`` and writes k/v to the paged cache.
    Returns strided views (q [T,Hq,hd], k [T,Hkv,hd], v [T,Hkv,hd]) into ``qkv``."""
    q, k, v = split_qkv(qkv, hq, hkv, hd)
    if use_rope:
        q.copy_(apply_rope(q, positions, cos_sin))
        k.copy_(apply_rope(k, positions, cos_sin))
    if k_cache is not None:
        write_kv(k, v, slot_mapping, k_cache, v_cache)
    return q, k, v


# ----------------------------------------------------------------------------- attention (K7, K8)
def prefill_attention(q, k, v, cu_seqlens: torch.Tensor, scale: float) -> torch.Tensor:
    """Causal varlen GQA attention. q [T,Hq,hd], k/v [T,Hkv,hd] -> [T,Hq,hd]."""
    out = torch.empty(q.shape, dtype=q.dtype, device=q.device)
    hq, hkv = q.shape[1], k.shape[1]
    rep = hq // hkv
    cu = cu_seqlens.tolist()
    for i in range(len(cu) - 1):
        s, e = cu[i], cu[i + 1]
        if e <= s:
            continue
        qs = q[s:e].float().transpose(0, 1)                   # [Hq, L, hd]
        ks = k[s:e].float().transpose(0, 1).repeat_interleave(rep, 0)
        vs = v[s:e].float().transpose(0, 1).repeat_interleave(rep, 0)
        sc = (qs @ ks.transpose(1, 2)) * scale
        L = e - s
        mask = torch.ones(L, L, dtype=torch.bool, device=q.device).triu(1)
        sc = sc.masked_fill(mask, float("-inf"))
        o = sc.softmax(-1) @ vs
        out[s:e] = o.transpose(0, 1).to(q.dtype)
    return out


def gather_kv(k_cache, v_cache, block_table: torch.Tensor, ctx_len: int):
    """Contiguous [ctx, Hkv, hd] K and V for one sequence from the paged cache."""
    bs = k_cache.shape[2]
    nblk = (ctx_len + bs - 1) // bs
    blocks = block_table[:nblk].long()
    kk = k_cache[blocks].permute(0, 2, 1, 3).reshape(nblk * bs, k_cache.shape[1], -1)[:ctx_len]
    vv = v_cache[blocks].permute(0, 2, 1, 3).reshape(nblk * bs, v_cache.shape[1], -1)[:ctx_len]
    return kk, vv


def prefill_attention_paged(q, k_cache, v_cache, cu_seqlens, context_lens, block_tables,
                            scale: float) -> torch.Tensor:
    """Chunked prefill: the queries q[cu[i]:cu[i+1]] sit at positions [ctx-L, ctx) of
    sequence i and attend causally over its ctx = context_lens[i] cached keys."""
    out = torch.empty(q.shape, dtype=q.dtype, device=q.device)
    hq, hkv = q.shape[1], k_cache.shape[1]
    rep = hq // hkv
    cu, lens = cu_seqlens.tolist(), context_lens.tolist()
    for i in range(len(cu) - 1):
        s, e = cu[i], cu[i + 1]
        if e <= s:
            continue
        L, ctx = e - s, lens[i]
        kk, vv = gather_kv(k_cache, v_cache, block_tables[i], ctx)
        kk = kk.float().transpose(0, 1).repeat_interleave(rep, 0)   # [Hq, ctx, hd]
        vv = vv.float().transpose(0, 1).repeat_interleave(rep, 0)
        qs = q[s:e].float().transpose(0, 1)                          # [Hq, L, hd]
        sc = (qs @ kk.transpose(1, 2)) * scale                       # [Hq, L, ctx]
        qpos = torch.arange(ctx - L, ctx, device=q.device).unsqueeze(1)
        mask = torch.arange(ctx, device=q.device).unsqueeze(0) > qpos
        sc = sc.masked_fill(mask, float("-inf"))
        out[s:e] = (sc.softmax(-1) @ vv).transpose(0, 1).to(q.dtype)
    return out


def decode_attention(q, k_cache, v_cache, block_tables, context_lens, scale) -> torch.Tensor:
    """q [B,Hq,hd] single query per sequence against its paged cache."""
    out = torch.empty(q.shape, dtype=q.dtype, device=q.device)
    hq, hkv = q.shape[1], k_cache.shape[1]
    rep = hq // hkv
    lens = context_lens.tolist()
    for b, L in enumerate(lens):
        if L <= 0:
            out[b] = 0
            continue
        kk, vv = gather_kv(k_cache, v_cache, block_tables[b], L)
        kk = kk.float().transpose(0, 1).repeat_interleave(rep, 0)   # [Hq, L, hd]
        vv = vv.float().transpose(0, 1).repeat_interleave(rep, 0)
        sc = (kk @ q[b].float().unsqueeze(-1)).squeeze(-1) * scale  # [Hq, L]
        out[b] = (sc.softmax(-1).unsqueeze(1) @ vv).squeeze(1).to(q.dtype)
    return out


# ----------------------------------------------------------------------------- sampling (K13)
def topk_topp_filter(logits: torch.Tensor, temperature: torch.Tensor, top_k: torch.Tensor,
                     top_p: torch.Tensor) -> torch.Tensor:
    """HF warper order: Temperature -> TopK (ties kept) -> TopP (min_tokens_to_keep=1).
    Returns filtered fp32 logits (-inf outside the support)."""
    x = logits.float() / temperature.float().clamp_min(1e-6)[:, None]
    out = torch.full_like(x, float("-inf"))
    for i in range(x.shape[0]):
        row = x[i]
        k = int(top_k[i])
        if 0 < k < row.numel():
            kth = torch.topk(row, k).values[-1]
            row = row.masked_fill(row < kth, float("-inf"))
        p = float(top_p[i])
        if p < 1.0:
            srt, idx = torch.sort(row, descending=False)
            cum = srt.softmax(-1).cumsum(-1)
            remove = cum <= (1 - p)
            remove[-1] = False
            row = row.clone()
            row[idx[remove]] = float("-inf")
        out[i] = row
    return out


def _draw(probs: torch.Tensor, ids: torch.Tensor, g: torch.Generator) -> int:
    """Inverse-CDF draw over the support ordered by (probability desc, token id asc): the
    token drawn depends only on (token id, probability) pairs, not on where they sit in the
    row, so sampling from a candidate list (vocab-parallel LM head) equals sampling from the
    full vocabulary (same contract as the HIP sampler's sorted inverse-CDF draw)."""
    nz = (probs > 0).nonzero().squeeze(-1)
    pv, iv = probs[nz].double(), ids[nz]
    o1 = torch.argsort(iv)
    pv, iv = pv[o1], iv[o1]
    o2 = torch.sort(-pv, stable=True).indices
    pv, iv = pv[o2], iv[o2]
    u = torch.rand((), generator=g, dtype=torch.float64) * pv.sum()
    j = int(torch.searchsorted(pv.cumsum(0), u, right=True).clamp_max(pv.numel() - 1))
    return int(iv[j])


def sample(logits: torch.Tensor, temperature: torch.Tensor, top_k: torch.Tensor,
           top_p: torch.Tensor, generator: Optional[torch.Generator] = None,
           seeds: Optional[torch.Tensor] = None,
           ids: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Returns int32 token ids [B]. temperature<=0 (or top_k == 1) -> greedy argmax (lowest
    token id on ties). ``ids`` [B, C]: the row holds candidates (vocab-parallel LM head)
    whose token ids are ``ids``; default ids = column index. With per-row ``seeds`` each row
    draws from its own generator, so a request's tokens do not depend on its batch
    neighbours (same contract as the HIP sampler)."""
    B, V = logits.shape
    if ids is None:
        ids = torch.arange(V, device=logits.device, dtype=torch.int64).expand(B, V)
    ids = ids.long()
    greedy = (temperature <= 0) | (top_k == 1)
    out = torch.empty(B, dtype=torch.int32, device=logits.device)
    x = logits.float()
    for r in greedy.nonzero().squeeze(-1).tolist():
        m = x[r] == x[r].max()
        out[r] = int(ids[r][m].min())
    ng = ~greedy
    if ng.any():
        rows = ng.nonzero().squeeze(-1).tolist()
        filt = topk_topp_filter(x[ng], temperature[ng], top_k[ng], top_p[ng])
        probs = filt.softmax(-1)
        sd = seeds.tolist() if seeds is not None else None
        for j, r in enumerate(rows):
            if sd is None:
                g = generator
                if g is None:
                    g = torch.Generator(device=probs.device)
                    g.seed()
            else:
                g = torch.Generator(device=probs.device)
                g.manual_seed(int(sd[r]) & 0x7FFF_FFFF_FFFF_FFFF)
            out[r] = _draw(probs[j], ids[r], g)
    return out


def head_candidates(h: torch.Tensor, w_slice: torch.Tensor, offset: int, c: int):
    """Vocab-parallel LM head slice: fp32 logits of rows ``[offset, offset + V_r)`` and
    their top-``c`` (values desc, token ids) -> (fp32 [S, c], int32 [S, c])."""
    lg = linear(h, w_slice, out_dtype=torch.float32)
    v, i = torch.topk(lg, min(c, lg.shape[1]), dim=-1)
    return v, (i + offset).to(torch.int32)


# ----------------------------------------------------------------------------- MoE (K15, K16)
def router_topk(router_logits: torch.Tensor, k: int):
    """Mixtral routing: softmax -> topk -> renormalise. Returns (weights fp32 [T,k], ids int32)."""
    p = router_logits.float().softmax(-1)
    w, ids = torch.topk(p, k, dim=-1)
    w = w / w.sum(-1, keepdim=True)
    return w, ids.to(torch.int32)


def moe_mlp(x: torch.Tensor, w_gu: torch.Tensor, w_down: torch.Tensor,
            topk_w: torch.Tensor, topk_ids: torch.Tensor,
            expert_offset: int = 0) -> torch.Tensor:
    """x [T,D]; w_gu [E_local, 2F, D] (interleaved); w_down [E_local, D, F].
    Only experts in [expert_offset, expert_offset+E_local) contribute (EP shard)."""
    t = x.shape[0]
    e_local = w_gu.shape[0]
    out = torch.zeros(t, x.shape[1], dtype=torch.float32, device=x.device)
    for le in range(e_local):
        e = le + expert_offset
        rows, slot = (topk_ids == e).nonzero(as_tuple=True)
        if rows.numel() == 0:
            continue
        h = silu_mul(linear(x[rows], w_gu[le]))
        y = linear(h, w_down[le]).float()
        out.index_add_(0, rows, y * topk_w[rows, slot][:, None])
    return out.to(x.dtype)
