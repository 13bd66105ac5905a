"""HF checkpoint import: ``save_pretrained`` directories (and hub-cache snapshots) of
LlamaForCausalLM / MixtralForCausalLM / GPT2LMHeadModel.

The reference loads checkpoints with ``AutoModelForCausalLM.from_pretrained(model_name,
cache_dir=MODEL_CACHE_DIR)`` (``worker/app.py:117-124``) and its sharder shards a loaded HF
model (``master/dashboard/management/commands/shard_model.py:37,55-96``). Here a checkpoint
directory is read without transformers at run time:

* ``config.json`` -> ``ModelConfig`` (``config_from_hf``);
* ``model.safetensors`` or ``model.safetensors.index.json`` + its shard files, read tensor by
  tensor through the C++ safetensors loader (mmap, no pickle) as ``from_hf_state_dict`` asks
  for them, so host memory holds the converted stage, not the checkpoint twice;
* ``layers`` / ``first`` / ``last`` select one pipeline stage's tensors (``shard-model
  --from-hf``, or a worker loading only its stage).

Directory forms accepted by ``find_hf_dir``: the directory itself, ``<root>/<name with / ->
_>/``, and the HF hub cache layout ``<root>/models--<org>--<name>/snapshots/<rev>/``.
"""
from __future__ import annotations

import json
from pathlib import Path
from typing import Dict, Iterable, Iterator, Optional, Tuple

import torch

from .configs import ModelConfig
from .weights import from_hf_state_dict


def is_hf_dir(d) -> bool:
    d = Path(d)
    cj = d / "config.json"
    if not cj.exists():
        return False
    try:
        c = json.loads(cj.read_text())
    except (OSError, ValueError):
        return False
    return "model_type" in c and ((d / "model.safetensors").exists()
                                  or (d / "model.safetensors.index.json").exists())


def find_hf_dir(root: str, name: str) -> Optional[Path]:
    """The HF checkpoint directory of ``name`` under ``root`` (see module docstring)."""
    r = Path(root)
    cands = [r / name.replace("/", "_"), r / name]
    hub = r / ("models--" + name.replace("/", "--"))
    snaps = hub / "snapshots"
    if snaps.is_dir():
        ref = hub / "refs" / "main"
        if ref.exists():
            cands.append(snaps / ref.read_text().strip())
        cands += sorted(snaps.iterdir(), key=lambda p: p.stat().st_mtime, reverse=True)
    for c in cands:
        if c.is_dir() and is_hf_dir(c):
            return c
    return None


def config_from_hf(c: dict, name: Optional[str] = None) -> ModelConfig:
    """Map a HF ``config.json`` (llama / mistral / mixtral / gpt2 model types)."""
    mt = c.get("model_type", "")
    name = name or c.get("_name_or_path") or mt
    if mt == "gpt2":
        d = int(c["n_embd"])
        return ModelConfig(
            name=name, arch="gpt2", hidden_size=d, num_layers=int(c["n_layer"]),
            num_heads=int(c["n_head"]), num_kv_heads=int(c["n_head"]),
            head_dim=d // int(c["n_head"]), intermediate_size=int(c.get("n_inner") or 4 * d),
            vocab_size=int(c["vocab_size"]), max_position=int(c.get("n_positions", 1024)),
            rope_theta=0.0, norm_eps=float(c.get("layer_norm_epsilon", 1e-5)),
            tie_embeddings=True, bos_token_id=int(c.get("bos_token_id", 50256)),
            eos_token_id=_eos(c, 50256))
    if mt not in ("llama", "mistral", "mixtral"):
        raise ValueError(f"unsupported HF model_type '{mt}' (llama, mistral, mixtral, gpt2)")
    d, nh = int(c["hidden_size"]), int(c["num_attention_heads"])
    rope = c.get("rope_theta")
    params = c.get("rope_parameters") or {}
    if rope is None:
        rope = params.get("rope_theta", 10000.0)
    # rope scaling (Llama-3.1 / 3.2 "llama3", "linear"): absorbed into the cos/sin table;
    # transformers 5 keeps it in rope_parameters, older configs in rope_scaling
    sc = dict(c.get("rope_scaling") or {})
    if not sc and params.get("rope_type", "default") not in ("default", None):
        sc = {k: v for k, v in params.items() if k != "rope_theta"}
    if sc:
        from ..ops.reference import rope_scaled_inv_freq
        import torch as _t
        rope_scaled_inv_freq(_t.ones(2, dtype=_t.float64), sc)     # refuse unknown types now
    max_pos = int(c.get("max_position_embeddings", 8192))
    # sliding-window attention (Mistral): full attention equals it while a sequence fits the
    # window, so the model's context is capped there instead of silently diverging past it
    sw = c.get("sliding_window")
    if sw and int(sw) < max_pos:
        import logging
        logging.getLogger(__name__).warning(
            "sliding_window=%s < max_position_embeddings=%s: context capped at the window "
            "(sliding-window attention is not implemented)", sw, max_pos)
        max_pos = int(sw)
    return ModelConfig(
        name=name, arch="llama", hidden_size=d, num_layers=int(c["num_hidden_layers"]),
        num_heads=nh, num_kv_heads=int(c.get("num_key_value_heads") or nh),
        head_dim=int(c.get("head_dim") or d // nh),
        intermediate_size=int(c["intermediate_size"]), vocab_size=int(c["vocab_size"]),
        max_position=max_pos, rope_theta=float(rope),
        rope_scaling=tuple(sorted((str(k), v) for k, v in sc.items()
                                  if isinstance(v, (int, float, str)))),
        norm_eps=float(c.get("rms_norm_eps", 1e-5)),
        num_experts=int(c.get("num_local_experts", 0)) if mt == "mixtral" else 0,
        top_k_experts=int(c.get("num_experts_per_tok", 2)),
        tie_embeddings=bool(c.get("tie_word_embeddings", False)),
        bos_token_id=int(c.get("bos_token_id") or 1), eos_token_id=_eos(c, 2))


def _eos(c: dict, default: int) -> int:
    e = c.get("eos_token_id", default)
    if isinstance(e, list):
        e = e[0] if e else default
    return int(default if e is None else e)


class LazyStateDict:
    """Mapping over every tensor of a (possibly multi-file) safetensors checkpoint; a tensor
    is read from disk (C++ loader, to host memory) when it is first asked for."""

    def __init__(self, d: Path):
        from ..runtime import SafetensorsFile
        self.dir = Path(d)
        idx = self.dir / "model.safetensors.index.json"
        if idx.exists():
            wm = json.loads(idx.read_text())["weight_map"]
            files = sorted(set(wm.values()))
        else:
            files = ["model.safetensors"]
            wm = None
        self._files = {f: SafetensorsFile(str(self.dir / f)) for f in files}
        self._where: Dict[str, str] = {}
        for f, st in self._files.items():
            for k in st.keys():
                self._where[k] = f
        if wm is not None:
            missing = [k for k in wm if k not in self._where]
            if missing:
                raise ValueError(f"{idx}: {len(missing)} indexed tensors missing, e.g. "
                                 f"{missing[0]}")

    def __contains__(self, k) -> bool:
        return k in self._where

    def __getitem__(self, k) -> torch.Tensor:
        f = self._where[k]
        return self._files[f].load([k])[k]

    def keys(self) -> Iterator[str]:
        return iter(self._where)

    def close(self) -> None:
        for st in self._files.values():
            st.close()


def load_hf_dir(d, device="cpu", dtype=torch.bfloat16, name: Optional[str] = None,
                layers: Optional[Iterable[int]] = None, first: bool = True,
                last: bool = True) -> Tuple[ModelConfig, Dict[str, torch.Tensor]]:
    """(config, our parameter dict on ``device``) from a HF checkpoint directory; with
    ``layers`` / ``first`` / ``last`` only that pipeline stage's tensors."""
    d = Path(d)
    cfg = config_from_hf(json.loads((d / "config.json").read_text()), name)
    sd = LazyStateDict(d)
    try:
        params = from_hf_state_dict(cfg, sd, layers=layers, first=first, last=last, dtype=dtype)
    finally:
        sd.close()
    dev = torch.device(device)
    if dev.type != "cpu":
        params = {k: v.to(dev, non_blocking=True) for k, v in params.items()}
        torch.cuda.synchronize(dev)
    return cfg, params
