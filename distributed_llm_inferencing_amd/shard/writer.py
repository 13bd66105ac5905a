"""Shard export / import in the reference's on-disk layout:

    <output_dir>/<model_name with '/' -> '_'>/
        tokenizer/                     (reference: shard_model.py:29-33)
        shard_<i>/model.safetensors    ONLY stage i's tensors (the reference saved a full-size,
                                       mostly random model per shard, shard_model.py:71)
        shard_<i>/config.json          our ModelConfig
        shard_<i>/metadata.json        {"model_name","shard_id","num_shards","start_layer",
                                        "end_layer" (inclusive),"total_layers"} + extensions

Export works for any registered architecture (the reference only handled GPT-2,
``shard_model.py:40-50``). Weights are either random-init (deterministic per tensor name, so
shard i holds exactly the slice the full model would) or a provided state dict (e.g.
converted from HF with ``models.weights.from_hf_state_dict``). Import goes through the C++
safetensors loader (mmap -> pinned ring -> hipMemcpyAsync).
"""
from __future__ import annotations

import json
import os
from pathlib import Path
from typing import Dict, List, Optional, Tuple

import torch

from ..models import weights as W
from ..models.configs import ModelConfig, get_config
from ..tokenizer import load_tokenizer
from .planner import StagePlan, plan_stages

DEFAULT_METADATA = {"num_shards": 1, "start_layer": 0, "end_layer": 0, "total_layers": 1}


def model_dir(output_dir: str, model_name: str) -> Path:
    return Path(output_dir) / model_name.replace("/", "_")


def export_shards(model_name: str, num_shards: int, output_dir: str = "model_shards",
                  policy: str = "even", seed: int = 0, params: Optional[Dict] = None,
                  dtype=torch.bfloat16, cfg: Optional[ModelConfig] = None,
                  log=print, hf_dir: Optional[str] = None) -> List[Path]:
    """``hf_dir``: shard a HF ``save_pretrained`` checkpoint (the reference's sharder loads
    the HF model, shard_model.py:37): each stage reads only its own tensors from it."""
    from safetensors.torch import save_file
    if hf_dir is not None:
        from ..models.hf import config_from_hf
        cfg = config_from_hf(json.loads((Path(hf_dir) / "config.json").read_text()),
                             model_name)
    cfg = cfg or get_config(model_name)
    plans = plan_stages(cfg, num_shards, policy)
    root = model_dir(output_dir, model_name)
    root.mkdir(parents=True, exist_ok=True)
    load_tokenizer(cfg, hf_dir).save_pretrained(str(root / "tokenizer"))
    paths = []
    for p in plans:
        log(f"Shard {p.shard_id} will contain layers {p.start_layer} to {p.end_layer - 1}")
        shapes = W.stage_param_shapes(cfg, p.start_layer, p.end_layer, p.first, p.last)
        if hf_dir is not None:
            from ..models.hf import load_hf_dir
            _, sd = load_hf_dir(hf_dir, "cpu", dtype, model_name,
                                layers=range(p.start_layer, p.end_layer), first=p.first,
                                last=p.last)
            missing = set(shapes) - set(sd)
            if missing:
                raise ValueError(f"{hf_dir}: stage {p.shard_id} lacks {sorted(missing)[:3]}")
            sd = {k: sd[k] for k in shapes}
        elif params is None:
            sd = W.random_init(shapes, "cpu", dtype, seed)
        else:
            sd = {k: params[k].to(dtype).contiguous() for k in shapes}
        d = root / f"shard_{p.shard_id}"
        d.mkdir(parents=True, exist_ok=True)
        save_file({k: v.contiguous() for k, v in sd.items()}, str(d / "model.safetensors"),
                  metadata={"format": "dli", "model": cfg.name})
        (d / "config.json").write_text(json.dumps(cfg.to_dict(), indent=2))
        (d / "metadata.json").write_text(
            json.dumps(p.to_metadata(model_name, len(plans), cfg.num_layers), indent=2))
        paths.append(d)
        log(f"Shard {p.shard_id} created successfully")
    return paths


def read_metadata(shard_path: str, model_name: str, shard_id: int) -> dict:
    mp = Path(shard_path) / "metadata.json"
    if mp.exists():
        return json.loads(mp.read_text())
    # reference default when metadata.json is absent (worker/app.py:182-189)
    return {"model_name": model_name, "shard_id": shard_id, **DEFAULT_METADATA}


def load_shard(shard_path: str, device="cpu") -> Tuple[ModelConfig, dict, Dict[str, torch.Tensor]]:
    """(config, metadata, this stage's tensors on `device`) for one exported shard."""
    from ..runtime import SafetensorsFile
    d = Path(shard_path)
    cfg = ModelConfig.from_dict(json.loads((d / "config.json").read_text()))
    meta = json.loads((d / "metadata.json").read_text())
    st = SafetensorsFile(str(d / "model.safetensors"))
    try:
        params = st.load(device=device)
    finally:
        st.close()
    return cfg, meta, params


def load_cached_model(cache_dir: str, model_name: str, device="cpu",
                      dtype: Optional[torch.dtype] = None):
    """Whole-model weights from the model cache, or None when the cache holds none:
    a HF checkpoint (``save_pretrained`` directory or hub-cache snapshot, ``models/hf.py``;
    the reference's ``from_pretrained(cache_dir=MODEL_CACHE_DIR)``, worker/app.py:117-124),
    ``<cache>/<model>/model.safetensors`` + our ``config.json``, or every ``shard_<i>/`` of
    an export (merged). Returns (config, params on `device`, tokenizer dir or None)."""
    from ..models.hf import find_hf_dir, load_hf_dir
    hf = find_hf_dir(cache_dir, model_name)
    if hf is not None:
        dev = torch.device(device)
        dt = dtype or (torch.bfloat16 if dev.type == "cuda" else torch.float32)
        cfg, params = load_hf_dir(hf, device, dt, model_name)
        tok = str(hf) if any((hf / f).exists() for f in ("tokenizer.json",
                                                         "tokenizer_config.json")) else None
        return cfg, params, tok
    root = model_dir(cache_dir, model_name)
    if not root.is_dir():
        return None
    tok = str(root / "tokenizer") if (root / "tokenizer").is_dir() else None
    if (root / "model.safetensors").exists() and (root / "config.json").exists():
        from ..runtime import SafetensorsFile
        cfg = ModelConfig.from_dict(json.loads((root / "config.json").read_text()))
        f = SafetensorsFile(str(root / "model.safetensors"))
        try:
            params = f.load(device=device)
        finally:
            f.close()
        return cfg, params, tok
    shards = sorted((d for d in root.glob("shard_*") if (d / "model.safetensors").exists()),
                    key=lambda d: int(d.name.split("_")[1]))
    if not shards:
        return None
    cfg, params, covered = None, {}, 0
    for d in shards:
        c, meta, p = load_shard(str(d), device=device)
        if int(meta["start_layer"]) != covered:
            raise ValueError(f"{root}: shard {d.name} starts at layer {meta['start_layer']}, "
                             f"expected {covered}")
        covered = int(meta["end_layer"]) + 1
        cfg = c
        params.update(p)
    if covered != cfg.num_layers:
        raise ValueError(f"{root}: shards cover {covered} of {cfg.num_layers} layers")
    return cfg, params, tok


def stage_plan_from_metadata(meta: dict) -> StagePlan:
    s, e = int(meta["start_layer"]), int(meta["end_layer"]) + 1
    return StagePlan(int(meta["shard_id"]), s, e, int(meta.get("weight_bytes", 0)), 0.0,
                     s == 0, e == int(meta["total_layers"]))


def main(argv=None):
    """``shard-model`` CLI (reference: ``python manage.py shard_model --model_name X
    --num_shards N [--output_dir D]``, shard_model.py:11-14)."""
    import argparse
    ap = argparse.ArgumentParser("dli shard-model")
    ap.add_argument("--model_name", "--model-name", required=True)
    ap.add_argument("--num_shards", "--num-shards", type=int, required=True)
    ap.add_argument("--output_dir", "--output-dir", default="model_shards")
    ap.add_argument("--policy", default="even", choices=["even", "hbm", "balanced"])
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--from-hf", "--from_hf", dest="from_hf", default=None,
                    help="shard this HF save_pretrained checkpoint directory instead of a "
                         "random init")
    ap.add_argument("--register", default=None,
                    help="master URL: register each shard (node ids via --nodes)")
    ap.add_argument("--nodes", default="", help="comma-separated node ids, one per shard")
    a = ap.parse_args(argv)
    print(f"Sharding model {a.model_name} into {a.num_shards} shards")
    paths = export_shards(a.model_name, a.num_shards, a.output_dir, a.policy, a.seed,
                          hf_dir=a.from_hf)
    print(f"Model {a.model_name} sharded successfully into {a.num_shards} shards")
    print(f"Shards are stored in {model_dir(a.output_dir, a.model_name)}")
    if a.register:
        import requests
        nodes = [int(x) for x in a.nodes.split(",") if x]
        for i, p in enumerate(paths):
            nid = nodes[i % len(nodes)] if nodes else 1
            requests.post(f"{a.register}/api/shards/register/",
                          data={"node_id": nid, "model_name": a.model_name, "shard_id": i,
                                "path": str(p), "is_loaded": 0}, timeout=10)


if __name__ == "__main__":
    main()
