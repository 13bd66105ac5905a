"""Architecture registry: every model family the framework serves.

The reference loads arbitrary HF checkpoints through ``AutoModelForCausalLM``
(``worker/app.py:121``); offline we define the architectures ourselves from the
public HF ``config.json`` values and random-init them.

Names accepted by ``get_config`` are case-insensitive and include the HF hub ids
the reference UI would send (``gpt2``, ``meta-llama/Meta-Llama-3-8B`` ...).
"""
from __future__ import annotations

from dataclasses import asdict, dataclass, replace
from typing import Optional


@dataclass(frozen=True)
class ModelConfig:
    name: str
    arch: str                 # "llama" (llama / mixtral family) or "gpt2"
    hidden_size: int
    num_layers: int
    num_heads: int
    num_kv_heads: int
    head_dim: int
    intermediate_size: int
    vocab_size: int
    max_position: int = 8192
    rope_theta: float = 500000.0
    norm_eps: float = 1e-5
    num_experts: int = 0      # 0 -> dense MLP
    top_k_experts: int = 2
    tie_embeddings: bool = False
    bos_token_id: int = 1
    eos_token_id: int = 2
    # HF ``rope_scaling`` as sorted (key, value) pairs: () = none; rope_type "llama3"
    # (Llama-3.1 / 3.2 checkpoints: low-frequency inv_freq rescaled) or "linear"
    rope_scaling: tuple = ()

    @property
    def is_moe(self) -> bool:
        return self.num_experts > 0

    @property
    def q_size(self) -> int:
        return self.num_heads * self.head_dim

    @property
    def kv_size(self) -> int:
        return self.num_kv_heads * self.head_dim

    @property
    def qkv_size(self) -> int:
        return self.q_size + 2 * self.kv_size

    def layer_param_count(self) -> int:
        d, f = self.hidden_size, self.intermediate_size
        if self.arch == "gpt2":
            # c_attn (d x 3d + 3d), c_proj (d x d + d), c_fc (d x f + f), mlp c_proj (f x d + d), 2 LN
            return d * 3 * d + 3 * d + d * d + d + d * f + f + f * d + d + 4 * d
        attn = d * self.qkv_size + self.q_size * d
        mlp = 3 * d * f
        if self.is_moe:
            mlp = self.num_experts * mlp + d * self.num_experts
        return attn + mlp + 2 * d

    def embed_param_count(self) -> int:
        n = self.vocab_size * self.hidden_size
        if self.arch == "gpt2":
            n += self.max_position * self.hidden_size
        return n

    def head_param_count(self) -> int:
        """final norm + lm_head (0 extra for tied embeddings)."""
        n = 2 * self.hidden_size if self.arch == "gpt2" else self.hidden_size
        if not self.tie_embeddings:
            n += self.vocab_size * self.hidden_size
        return n

    def param_count(self) -> int:
        return (self.embed_param_count() + self.num_layers * self.layer_param_count()
                + self.head_param_count())

    def kv_bytes_per_token(self, dtype_bytes: int = 2) -> int:
        return 2 * self.num_layers * self.kv_size * dtype_bytes

    def to_dict(self) -> dict:
        return asdict(self)

    @classmethod
    def from_dict(cls, d: dict) -> "ModelConfig":
        fields = cls.__dataclass_fields__.keys()
        kw = {k: v for k, v in d.items() if k in fields}
        if "rope_scaling" in kw:         # JSON turned the pairs into lists
            kw["rope_scaling"] = tuple(tuple(p) for p in (kw["rope_scaling"] or ()))
        return cls(**kw)


GPT2 = ModelConfig(
    name="gpt2", arch="gpt2", hidden_size=768, num_layers=12, num_heads=12, num_kv_heads=12,
    head_dim=64, intermediate_size=3072, vocab_size=50257, max_position=1024, norm_eps=1e-5,
    tie_embeddings=True, bos_token_id=50256, eos_token_id=50256, rope_theta=0.0)

LLAMA3_8B = ModelConfig(
    name="llama3-8b", arch="llama", hidden_size=4096, num_layers=32, num_heads=32, num_kv_heads=8,
    head_dim=128, intermediate_size=14336, vocab_size=128256, max_position=8192,
    rope_theta=500000.0, norm_eps=1e-5, bos_token_id=128000, eos_token_id=128001)

LLAMA3_70B = replace(LLAMA3_8B, name="llama3-70b", hidden_size=8192, num_layers=80,
                     num_heads=64, num_kv_heads=8, intermediate_size=28672)

MIXTRAL_8X7B = ModelConfig(
    name="mixtral-8x7b", arch="llama", hidden_size=4096, num_layers=32, num_heads=32,
    num_kv_heads=8, head_dim=128, intermediate_size=14336, vocab_size=32000,
    max_position=32768, rope_theta=1e6, norm_eps=1e-5, num_experts=8, top_k_experts=2,
    bos_token_id=1, eos_token_id=2)

# Tiny variants: same code paths, test-sized. Shapes keep the hardware-friendly
# multiples (head_dim 64/128, hidden multiple of 256) so HIP kernels see real layouts.
LLAMA_TINY = ModelConfig(
    name="llama-tiny", arch="llama", hidden_size=256, num_layers=4, num_heads=4, num_kv_heads=2,
    head_dim=64, intermediate_size=512, vocab_size=1024, max_position=2048,
    rope_theta=10000.0, bos_token_id=1, eos_token_id=2)

LLAMA_TINY128 = replace(LLAMA_TINY, name="llama-tiny128", hidden_size=512, num_heads=4,
                        num_kv_heads=2, head_dim=128, intermediate_size=1024)

# 8 layers: one per stage of an 8-rank pipeline test
LLAMA_TINY8 = replace(LLAMA_TINY, name="llama-tiny8", num_layers=8)

MIXTRAL_TINY = replace(LLAMA_TINY, name="mixtral-tiny", num_experts=4, top_k_experts=2,
                       intermediate_size=256)

# 8 experts: one per rank of an 8-rank expert-parallel test
MIXTRAL_TINY8E = replace(MIXTRAL_TINY, name="mixtral-tiny8e", num_experts=8)

GPT2_TINY = replace(GPT2, name="gpt2-tiny", hidden_size=256, num_layers=2, num_heads=4,
                    num_kv_heads=4, head_dim=64, intermediate_size=1024, vocab_size=1024,
                    max_position=256, bos_token_id=1023, eos_token_id=1023)

_REGISTRY = {c.name: c for c in
             (GPT2, LLAMA3_8B, LLAMA3_70B, MIXTRAL_8X7B, LLAMA_TINY, LLAMA_TINY128,
              LLAMA_TINY8, MIXTRAL_TINY, MIXTRAL_TINY8E, GPT2_TINY)}

_ALIASES = {
    "openai-community/gpt2": "gpt2",
    "meta-llama/meta-llama-3-8b": "llama3-8b",
    "meta-llama/llama-3.1-8b": "llama3-8b",
    "meta-llama/meta-llama-3-8b-instruct": "llama3-8b",
    "llama-3-8b": "llama3-8b",
    "llama3_8b": "llama3-8b",
    "meta-llama/meta-llama-3-70b": "llama3-70b",
    "llama-3-70b": "llama3-70b",
    "llama3_70b": "llama3-70b",
    "mistralai/mixtral-8x7b-v0.1": "mixtral-8x7b",
    "mixtral": "mixtral-8x7b",
    "mixtral_8x7b": "mixtral-8x7b",
}


def list_models() -> list[str]:
    return sorted(_REGISTRY)


def get_config(name: str, num_layers: Optional[int] = None) -> ModelConfig:
    key = name.strip().lower()
    key = _ALIASES.get(key, key)
    if key not in _REGISTRY:
        raise KeyError(f"unknown model '{name}'; known: {', '.join(list_models())}")
    cfg = _REGISTRY[key]
    if num_layers is not None:
        cfg = replace(cfg, num_layers=num_layers)
    return cfg


def register(cfg: ModelConfig) -> None:
    _REGISTRY[cfg.name] = cfg
