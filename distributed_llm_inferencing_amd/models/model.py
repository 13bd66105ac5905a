"""Transformer decoder for the Llama-3 / Mixtral / GPT-2 families, pipeline-stage aware.

One ``TransformerLM`` instance owns layers ``[layer_start, layer_end)`` of a model plus the
embedding (first stage) and final norm + LM head + sampler (last stage). It is the
replacement for the HF ``AutoModelForCausalLM.forward`` + ``generate`` hot loop the
reference worker runs (``worker/app.py:297-305``), re-built on our ops:

    embed -> [ (add_)rmsnorm -> QKV GEMM -> RoPE+KV write -> attention -> O GEMM
              -> add_rmsnorm -> gate/up GEMM with fused SiLU*mul -> down GEMM ] x L
          -> add_rmsnorm -> LM head (last token of each sequence, fp32) -> sampler

The residual add of every sub-block is fused into the next norm; at a stage boundary the
pending residual add is materialised so exactly one [T, D] tensor crosses the link.
MoE layers (Mixtral) route through ``self.moe_fn`` (local grouped GEMMs, or the
expert-parallel all-to-all implementation installed by ``parallel/expert.py``).
"""
from __future__ import annotations

import math
from typing import Callable, Dict, List, Optional, Tuple

import torch

from .. import ops
from ..engine.batch import DeviceBatch
from ..ops import reference as R
from .configs import ModelConfig
from . import weights as W


class TransformerLM:
    def __init__(self, cfg: ModelConfig, params: Dict[str, torch.Tensor], layer_start: int = 0,
                 layer_end: Optional[int] = None, device="cpu",
                 expert_range: Optional[Tuple[int, int]] = None):
        self.cfg = cfg
        self.layer_start = layer_start
        self.layer_end = cfg.num_layers if layer_end is None else layer_end
        self.is_first = layer_start == 0
        self.is_last = self.layer_end == cfg.num_layers
        self.device = torch.device(device)
        self.params = params
        self.expert_range = expert_range or ((0, cfg.num_experts) if cfg.is_moe else None)
        self.scale = 1.0 / math.sqrt(cfg.head_dim)
        self.cos_sin = None
        if cfg.arch == "llama":
            self.cos_sin = R.rope_cos_sin(cfg.max_position, cfg.head_dim, cfg.rope_theta,
                                          device=self.device, scaling=cfg.rope_scaling)
        self.moe_fn: Callable = self._moe_local
        # tensor-parallel mode (parallel/tensor.py): all-reduce(sum) of the row-parallel
        # O / down projections before their residual add
        self.tp_reduce: Optional[Callable] = None
        # vocab-parallel LM head (parallel/pipeline.py): the last stage returns the final
        # normed hidden state; every stage holds a vocab slice of the head
        self.vocab_parallel = False
        self.vocab_offset = 0
        self.layers = [self._layer_params(i) for i in range(self.layer_start, self.layer_end)]

    # ------------------------------------------------------------------ construction
    @classmethod
    def random(cls, cfg: ModelConfig, layer_start=0, layer_end=None, device="cpu",
               dtype=torch.bfloat16, seed=0, expert_range=None) -> "TransformerLM":
        le = cfg.num_layers if layer_end is None else layer_end
        shapes = W.stage_param_shapes(cfg, layer_start, le, layer_start == 0,
                                      le == cfg.num_layers, None)
        params = W.random_init(shapes, device, dtype, seed)
        if expert_range is not None:
            params = {k: W.slice_experts(k, v, expert_range) for k, v in params.items()}
        return cls(cfg, params, layer_start, le, device, expert_range)

    def _layer_params(self, i: int) -> dict:
        pre = f"layers.{i}."
        return {k[len(pre):]: v for k, v in self.params.items() if k.startswith(pre)}

    def param_bytes(self) -> int:
        return W.nbytes(self.params)

    def to(self, device):
        self.params = {k: v.to(device) for k, v in self.params.items()}
        self.device = torch.device(device)
        if self.cos_sin is not None:
            self.cos_sin = self.cos_sin.to(device)
        self.layers = [self._layer_params(i) for i in range(self.layer_start, self.layer_end)]
        return self

    # ------------------------------------------------------------------ forward
    def embed(self, b: DeviceBatch) -> torch.Tensor:
        p = self.params
        if self.cfg.arch == "gpt2":
            return ops.embedding(b.input_ids, p["embed"], p["pos_embed"], b.positions)
        return ops.embedding(b.input_ids, p["embed"])

    def forward_layers(self, x: torch.Tensor, b: DeviceBatch,
                       kv_caches: List[Tuple[torch.Tensor, torch.Tensor]]) -> torch.Tensor:
        """Runs this stage's layers; returns the hidden state with the residual folded in."""
        cfg = self.cfg
        if cfg.arch != "gpt2":
            return self._llama_layers(x, b, kv_caches)
        residual = torch.empty_like(x)
        pending = None             # output of the previous sub-block awaiting its residual add
        for li, lp in enumerate(self.layers):
            kc, vc = kv_caches[li] if kv_caches else (None, None)
            if cfg.arch == "gpt2":
                h = (ops.layernorm(x, lp["ln1_w"], lp["ln1_b"], cfg.norm_eps, residual_copy=residual)
                     if pending is None else
                     ops.add_layernorm(pending, residual, lp["ln1_w"], lp["ln1_b"], cfg.norm_eps))
                qkv = ops.linear(h, lp["wqkv"], lp["bqkv"])
            else:
                h = (ops.rmsnorm(x, lp["attn_norm"], cfg.norm_eps, residual_copy=residual)
                     if pending is None else
                     ops.add_rmsnorm(pending, residual, lp["attn_norm"], cfg.norm_eps))
                qkv = ops.linear(h, lp["wqkv"])
            attn = self._attention(qkv, b, kc, vc)
            if cfg.arch == "gpt2":
                o = ops.linear(attn, lp["wo"], lp["bo"])
                h = ops.add_layernorm(o, residual, lp["ln2_w"], lp["ln2_b"], cfg.norm_eps)
                f = ops.linear(h, lp["w_fc"], lp["b_fc"], epi="bias_gelu")
                pending = ops.linear(f, lp["w_proj"], lp["b_proj"])
            else:
                o = ops.linear(attn, lp["wo"])
                h = ops.add_rmsnorm(o, residual, lp["mlp_norm"], cfg.norm_eps)
                if cfg.is_moe:
                    pending = self.moe_fn(h, lp, self.layer_start + li)
                else:
                    act = ops.linear(h, lp["w_gu"], epi="silu_mul")
                    pending = ops.linear(act, lp["w_down"])
        if pending is None:
            return x
        residual.add_(pending)
        return residual

    def _llama_layers(self, x: torch.Tensor, b: DeviceBatch, kv_caches) -> torch.Tensor:
        """Llama / Mixtral layers with the split-K reduces fused into their consumers:
        QKV GEMM -> (reduce + RoPE + KV write), O GEMM -> (reduce + residual add + RMSNorm),
        down GEMM -> (reduce + residual add + NEXT layer's input RMSNorm)."""
        cfg = self.cfg
        eps = cfg.norm_eps
        residual = torch.empty_like(x)
        n = len(self.layers)
        if n == 0:
            return x
        h = ops.rmsnorm(x, self.layers[0]["attn_norm"], eps, residual_copy=residual)
        pending = None
        # batch-1 / tiny decode steps: the O and down GEMVs add into the residual themselves
        # and the next GEMV normalises its input rows in its prologue (ops.NormedRows), so no
        # split-K reduce + RMSNorm kernel runs between them (2 kernels fewer per layer)
        defer = (not b.is_prefill and self.tp_reduce is None and not cfg.is_moe
                 and ops.deferred_norm_ok(x))
        for li, lp in enumerate(self.layers):
            kc, vc = kv_caches[li] if kv_caches else (None, None)
            if pending is not None:          # MoE output of the previous layer
                h = ops.add_rmsnorm(pending, residual, lp["attn_norm"], eps)
                pending = None
            attn = None
            if not b.is_prefill:             # decode: reduce + RoPE + KV write + attention fused
                attn = ops.linear_rope_attention(h, lp["wqkv"], b.positions, b.slot_mapping,
                                                 self.cos_sin, kc, vc, b.block_tables,
                                                 b.context_lens, b.max_context, cfg.num_heads,
                                                 cfg.num_kv_heads, cfg.head_dim, self.scale)
            if attn is None:
                qkv = ops.linear_rope_cache(h, lp["wqkv"], b.positions, b.slot_mapping,
                                            self.cos_sin, kc, vc, cfg.num_heads,
                                            cfg.num_kv_heads, cfg.head_dim)
                attn = self._attend(qkv, b, kc, vc)
            if cfg.is_moe and self.tp_reduce is None and not defer:
                # O projection + add + RMSNorm with the MoE gate of its output rows (one
                # kernel when the slabs allow: ops.linear_add_rmsnorm route)
                h, tw, ti = ops.linear_add_rmsnorm(attn, lp["wo"], residual, lp["mlp_norm"],
                                                   eps, route=(lp["router"],
                                                               cfg.top_k_experts))
                pending = self.moe_fn(h, lp, self.layer_start + li, (tw, ti))
                continue
            h = self._proj_add_norm(attn, lp["wo"], residual, lp["mlp_norm"], eps, defer)
            if cfg.is_moe:
                pending = self.moe_fn(h, lp, self.layer_start + li)
                continue
            act = ops.linear(h, lp["w_gu"], epi="silu_mul")
            nxt = self.layers[li + 1]["attn_norm"] if li + 1 < n else None
            h = self._proj_add_norm(act, lp["w_down"], residual, nxt, eps, defer)
        if pending is not None:
            if isinstance(pending, ops.MoEPending):
                pending.add_rmsnorm(residual, None, eps)
            else:
                residual.add_(pending)
        return residual

    def _proj_add_norm(self, x, w, residual, norm_w, eps, defer: bool = False):
        if defer:
            ops.linear_residual(x, w, residual)
            return None if norm_w is None else ops.NormedRows(residual, norm_w, eps)
        if self.tp_reduce is None:
            return ops.linear_add_rmsnorm(x, w, residual, norm_w, eps)
        y = self.tp_reduce(ops.linear(x, w))
        if norm_w is None:
            residual.add_(y)
            return None
        return ops.add_rmsnorm(y, residual, norm_w, eps)

    def _attend(self, qkv, b: DeviceBatch, kc, vc) -> torch.Tensor:
        cfg = self.cfg
        if b.is_prefill:
            if b.num_decode:                     # mixed step: decode rows, then prefill chunks
                nd = b.num_decode
                out = torch.empty(qkv.shape[0], cfg.num_heads * cfg.head_dim,
                                  dtype=qkv.dtype, device=qkv.device)
                ops.decode_attention(qkv[:nd], kc, vc, b.block_tables[:nd],
                                     b.context_lens[:nd], b.max_context_decode, cfg.num_heads,
                                     cfg.num_kv_heads, cfg.head_dim, self.scale, out=out[:nd])
                ops.prefill_attention_paged(qkv[nd:], b.cu_seqlens_prefill,
                                            b.max_seqlen_prefill, b.context_lens[nd:],
                                            b.block_tables[nd:], kc, vc, cfg.num_heads,
                                            cfg.num_kv_heads, cfg.head_dim, self.scale,
                                            out=out[nd:])
                return out
            if b.block_tables is not None:       # chunked prefill over the paged cache
                return ops.prefill_attention_paged(qkv, b.cu_seqlens, b.max_seqlen,
                                                   b.context_lens, b.block_tables, kc, vc,
                                                   cfg.num_heads, cfg.num_kv_heads,
                                                   cfg.head_dim, self.scale)
            return ops.prefill_attention(qkv, b.cu_seqlens, b.max_seqlen, cfg.num_heads,
                                         cfg.num_kv_heads, cfg.head_dim, self.scale)
        return ops.decode_attention(qkv, kc, vc, b.block_tables, b.context_lens, b.max_context,
                                    cfg.num_heads, cfg.num_kv_heads, cfg.head_dim, self.scale)

    def _attention(self, qkv, b: DeviceBatch, kc, vc) -> torch.Tensor:
        cfg = self.cfg
        ops.rope_and_cache(qkv, b.positions, b.slot_mapping, self.cos_sin, kc, vc, cfg.num_heads,
                           cfg.num_kv_heads, cfg.head_dim, use_rope=cfg.arch != "gpt2")
        return self._attend(qkv, b, kc, vc)

    def _moe_local(self, h: torch.Tensor, lp: dict, layer: int, routing=None):
        """The layer's experts on this device. With ``routing`` (the gate computed in the O
        projection's reduce, ``_llama_layers``) a decode step returns an ``ops.MoEPending``:
        its combine runs inside the next layer's add + RMSNorm."""
        topk_w, topk_ids = (routing if routing is not None
                            else ops.moe_router(h, lp["router"], self.cfg.top_k_experts))
        e0 = self.expert_range[0] if self.expert_range else 0
        return ops.moe_mlp(h, lp["w_gu"], lp["w_down"], topk_w, topk_ids, e0,
                           defer_combine=routing is not None)

    def final_hidden(self, hidden: torch.Tensor, b: DeviceBatch) -> torch.Tensor:
        """Final norm of the last token of each sequence -> bf16 [S, D]."""
        cfg, p = self.cfg, self.params
        if b.is_prefill:
            hidden = hidden.index_select(0, b.last_token_idx)
        if cfg.arch == "gpt2":
            return ops.layernorm(hidden, p["final_norm"], p["final_norm_b"], cfg.norm_eps)
        return ops.rmsnorm(hidden, p["final_norm"], cfg.norm_eps)

    def head_logits(self, h: torch.Tensor) -> torch.Tensor:
        """LM head with fp32 logits (``ops.HEAD_EPI``: the GEMM's fp32 accumulators stored as
        they are); the sampler compares their exact values."""
        p = self.params
        return ops.linear(h, p["embed"] if self.cfg.tie_embeddings else p["lm_head"],
                          epi=ops.HEAD_EPI)

    def logits(self, hidden: torch.Tensor, b: DeviceBatch) -> torch.Tensor:
        """Final norm + LM head on the last token of each sequence -> [S, V] logits."""
        return self.head_logits(self.final_hidden(hidden, b))

    def head_candidates(self, h: torch.Tensor, c: int = 64):
        """This rank's slice of a vocab-parallel LM head (``params['head_slice']`` = rows
        ``[vocab_offset, vocab_offset + V_r)``): top-``c`` (fp32 values, int32 ids)."""
        return ops.head_candidates(h, self.params["head_slice"], self.vocab_offset, c)

    def sample(self, logits: torch.Tensor, b: DeviceBatch, generator=None) -> torch.Tensor:
        return ops.sample(logits, b.temperature, b.top_k, b.top_p, b.seeds, generator=generator)

    def forward(self, b: DeviceBatch, kv_caches, hidden: Optional[torch.Tensor] = None,
                return_logits: bool = False):
        """Stage forward. First stage embeds ``b.input_ids``; otherwise ``hidden`` is the
        previous stage's output. Last stage returns sampled int32 tokens [S] (and the logits
        when asked); other stages return the hidden state [T, D]."""
        x = self.embed(b) if self.is_first else hidden
        x = self.forward_layers(x, b, kv_caches)
        if not self.is_last:
            return x
        if self.vocab_parallel:          # the LM head runs sliced on every pipeline rank
            return self.final_hidden(x, b)
        lg = self.logits(x, b)
        tok = self.sample(lg, b)
        return (tok, lg) if return_logits else tok
