"""Weight naming, random init, HF-layout conversion and per-stage selection.

Our in-memory layout (all [out, in] row-major like torch Linear, bf16):

llama / mixtral (per layer ``layers.{i}.``):
    attn_norm [D], wqkv [(Hq+2Hkv)*hd, D], wo [D, Hq*hd], mlp_norm [D],
    dense: w_gu [2F, D] (16-row gate/up interleave, see ops/reference.py), w_down [D, F]
    moe:   router [E, D], w_gu [E, 2F, D], w_down [E, D, F]
gpt2 (per layer): ln1_w, ln1_b, wqkv [3D, D], bqkv [3D], wo [D, D], bo [D], ln2_w, ln2_b,
    w_fc [F, D], b_fc [F], w_proj [D, F], b_proj [D]
globals: embed [V, D], (gpt2) pos_embed [P, D], final_norm [D], (gpt2) final_norm_b [D],
    lm_head [V, D] (absent when tied to embed)

Random init mirrors HF ``_init_weights`` (normal(0, 0.02), norms = 1, biases = 0) and is
generated directly on the target device, per stage, so a 70B stage never materialises the
full model anywhere.
"""
from __future__ import annotations

from typing import Dict, Iterable, Optional

import torch

from .configs import ModelConfig
from ..ops.reference import interleave_gate_up

INIT_STD = 0.02


def layer_param_shapes(cfg: ModelConfig, i: int) -> Dict[str, tuple]:
    d, f, hd = cfg.hidden_size, cfg.intermediate_size, cfg.head_dim
    p = f"layers.{i}."
    if cfg.arch == "gpt2":
        return {p + "ln1_w": (d,), p + "ln1_b": (d,), p + "wqkv": (3 * d, d), p + "bqkv": (3 * d,),
                p + "wo": (d, d), p + "bo": (d,), p + "ln2_w": (d,), p + "ln2_b": (d,),
                p + "w_fc": (f, d), p + "b_fc": (f,), p + "w_proj": (d, f), p + "b_proj": (d,)}
    s = {p + "attn_norm": (d,), p + "wqkv": (cfg.qkv_size, d), p + "wo": (d, cfg.q_size),
         p + "mlp_norm": (d,)}
    if cfg.is_moe:
        e = cfg.num_experts
        s.update({p + "router": (e, d), p + "w_gu": (e, 2 * f, d), p + "w_down": (e, d, f)})
    else:
        s.update({p + "w_gu": (2 * f, d), p + "w_down": (d, f)})
    return s


def global_param_shapes(cfg: ModelConfig, first: bool, last: bool) -> Dict[str, tuple]:
    d, v = cfg.hidden_size, cfg.vocab_size
    s: Dict[str, tuple] = {}
    if first or (last and cfg.tie_embeddings):
        s["embed"] = (v, d)
    if first and cfg.arch == "gpt2":
        s["pos_embed"] = (cfg.max_position, d)
    if last:
        s["final_norm"] = (d,)
        if cfg.arch == "gpt2":
            s["final_norm_b"] = (d,)
        if not cfg.tie_embeddings:
            s["lm_head"] = (v, d)
    return s


def stage_param_shapes(cfg: ModelConfig, layer_start: int, layer_end: int, first: bool,
                       last: bool, expert_range: Optional[tuple] = None) -> Dict[str, tuple]:
    s = global_param_shapes(cfg, first, last)
    for i in range(layer_start, layer_end):
        ls = layer_param_shapes(cfg, i)
        if expert_range is not None and cfg.is_moe:
            e0, e1 = expert_range
            for k in list(ls):
                if k.endswith(".w_gu") or k.endswith(".w_down"):
                    ls[k] = (e1 - e0,) + tuple(ls[k][1:])
        s.update(ls)
    return s


def _is_norm_weight(name: str) -> bool:
    return name.endswith(("attn_norm", "mlp_norm", "final_norm", "ln1_w", "ln2_w"))


def _is_bias(name: str) -> bool:
    return name.endswith(("ln1_b", "ln2_b", "bqkv", "bo", "b_fc", "b_proj", "final_norm_b"))


def random_init(shapes: Dict[str, tuple], device, dtype=torch.bfloat16, seed: int = 0,
                std: float = INIT_STD) -> Dict[str, torch.Tensor]:
    """Deterministic per-tensor init: each tensor's values depend only on (seed, name), so a
    pipeline stage generates exactly the slice the full model would hold."""
    out = {}
    dev = torch.device(device)
    for name in sorted(shapes):
        shape = shapes[name]
        if _is_norm_weight(name):
            out[name] = torch.ones(shape, dtype=dtype, device=dev)
        elif _is_bias(name):
            out[name] = torch.zeros(shape, dtype=dtype, device=dev)
        else:
            g = torch.Generator(device=dev)
            g.manual_seed((seed * 1_000_003 + _name_hash(name)) & 0x7FFF_FFFF_FFFF)
            t = torch.empty(shape, dtype=dtype, device=dev)
            t.normal_(0.0, std, generator=g)
            out[name] = t
    return out


def slice_experts(name: str, t: torch.Tensor, expert_range: Optional[tuple]) -> torch.Tensor:
    if expert_range is None or not (name.endswith(".w_gu") or name.endswith(".w_down")):
        return t
    if t.dim() != 3:
        return t
    if expert_range[0] == 0 and expert_range[1] == t.shape[0]:
        return t
    # a copy: a leading-dim slice is already contiguous, so .contiguous() would return a
    # view that keeps every expert's storage alive (each EP rank held all 8 experts)
    return t[expert_range[0]:expert_range[1]].clone()


def _name_hash(name: str) -> int:
    h = 1469598103934665603
    for ch in name.encode():
        h ^= ch
        h = (h * 1099511628211) & 0xFFFF_FFFF_FFFF_FFFF
    return h


def nbytes(params: Dict[str, torch.Tensor]) -> int:
    return sum(t.numel() * t.element_size() for t in params.values())


# ----------------------------------------------------------------------------- HF conversion
def from_hf_state_dict(cfg: ModelConfig, sd: Dict[str, torch.Tensor],
                       layers: Optional[Iterable[int]] = None, first: bool = True,
                       last: bool = True, dtype=torch.bfloat16) -> Dict[str, torch.Tensor]:
    """Convert a HF LlamaForCausalLM / MixtralForCausalLM / GPT2LMHeadModel state dict."""
    layers = range(cfg.num_layers) if layers is None else layers
    out: Dict[str, torch.Tensor] = {}
    cv = lambda t: t.detach().to(dtype).contiguous()  # noqa: E731
    if cfg.arch == "gpt2":
        pre = "transformer."
        if first or (last and cfg.tie_embeddings):
            out["embed"] = cv(sd[pre + "wte.weight"])
        if first:
            out["pos_embed"] = cv(sd[pre + "wpe.weight"])
        if last:
            out["final_norm"] = cv(sd[pre + "ln_f.weight"])
            out["final_norm_b"] = cv(sd[pre + "ln_f.bias"])
        for i in layers:
            h = f"{pre}h.{i}."
            p = f"layers.{i}."
            # HF GPT-2 Conv1D stores [in, out]; ours is [out, in]
            out[p + "ln1_w"] = cv(sd[h + "ln_1.weight"]); out[p + "ln1_b"] = cv(sd[h + "ln_1.bias"])
            out[p + "wqkv"] = cv(sd[h + "attn.c_attn.weight"].t()); out[p + "bqkv"] = cv(sd[h + "attn.c_attn.bias"])
            out[p + "wo"] = cv(sd[h + "attn.c_proj.weight"].t()); out[p + "bo"] = cv(sd[h + "attn.c_proj.bias"])
            out[p + "ln2_w"] = cv(sd[h + "ln_2.weight"]); out[p + "ln2_b"] = cv(sd[h + "ln_2.bias"])
            out[p + "w_fc"] = cv(sd[h + "mlp.c_fc.weight"].t()); out[p + "b_fc"] = cv(sd[h + "mlp.c_fc.bias"])
            out[p + "w_proj"] = cv(sd[h + "mlp.c_proj.weight"].t()); out[p + "b_proj"] = cv(sd[h + "mlp.c_proj.bias"])
        return out
    if first:
        out["embed"] = cv(sd["model.embed_tokens.weight"])
    if last:
        out["final_norm"] = cv(sd["model.norm.weight"])
        if cfg.tie_embeddings:
            out["embed"] = cv(sd["model.embed_tokens.weight"])
        else:
            out["lm_head"] = cv(sd["lm_head.weight"])
    for i in layers:
        h = f"model.layers.{i}."
        p = f"layers.{i}."
        out[p + "attn_norm"] = cv(sd[h + "input_layernorm.weight"])
        out[p + "mlp_norm"] = cv(sd[h + "post_attention_layernorm.weight"])
        out[p + "wqkv"] = cv(torch.cat([sd[h + "self_attn.q_proj.weight"],
                                        sd[h + "self_attn.k_proj.weight"],
                                        sd[h + "self_attn.v_proj.weight"]], 0))
        out[p + "wo"] = cv(sd[h + "self_attn.o_proj.weight"])
        if cfg.is_moe:
            moe = h + "block_sparse_moe."
            if moe + "gate.weight" not in sd:
                moe = h + "mlp."
            out[p + "router"] = cv(sd[moe + "gate.weight"])
            gus, downs = [], []
            if moe + "experts.gate_up_proj" in sd:
                # fused expert tensors (transformers >= 5 MixtralExperts):
                # gate_up_proj [E, 2F, D] (gate rows then up rows), down_proj [E, D, F]
                gu = sd[moe + "experts.gate_up_proj"]
                dn = sd[moe + "experts.down_proj"]
                f = cfg.intermediate_size
                gus = [interleave_gate_up(gu[e, :f], gu[e, f:]) for e in range(cfg.num_experts)]
                downs = [dn[e] for e in range(cfg.num_experts)]
            else:
                for e in range(cfg.num_experts):
                    ex = f"{moe}experts.{e}."
                    if ex + "w1.weight" in sd:   # original Mixtral naming (w1 gate, w3 up, w2 down)
                        g, u, dn = sd[ex + "w1.weight"], sd[ex + "w3.weight"], sd[ex + "w2.weight"]
                    else:
                        g, u, dn = (sd[ex + "gate_proj.weight"], sd[ex + "up_proj.weight"],
                                    sd[ex + "down_proj.weight"])
                    gus.append(interleave_gate_up(g, u))
                    downs.append(dn)
            out[p + "w_gu"] = cv(torch.stack(gus))
            out[p + "w_down"] = cv(torch.stack(downs))
        else:
            out[p + "w_gu"] = cv(interleave_gate_up(sd[h + "mlp.gate_proj.weight"],
                                                    sd[h + "mlp.up_proj.weight"]))
            out[p + "w_down"] = cv(sd[h + "mlp.down_proj.weight"])
    return out
