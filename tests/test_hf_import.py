"""HF checkpoint import (models/hf.py): the reference loads checkpoints with
``from_pretrained(model_name, cache_dir=MODEL_CACHE_DIR)`` (worker/app.py:117-124) and shards a
loaded HF model (shard_model.py:37,55-96). Tiny random Llama / Mixtral / GPT-2 models are
written with transformers' ``save_pretrained`` (safetensors) and must come back through

* ``load_hf_dir``: last-position logits equal HF's (fp32);
* the worker's ``/load_model`` (MODEL_CACHE_DIR, plain and hub-cache layouts): greedy tokens
  equal HF ``generate``;
* ``shard-model --from-hf`` -> ``/load_shard`` -> sharded ``/inference``: the same tokens.
"""
import json
import os

import pytest
import torch

from distributed_llm_inferencing_amd.config import Settings
from distributed_llm_inferencing_amd.models import get_config
from distributed_llm_inferencing_amd.models.hf import config_from_hf, find_hf_dir, load_hf_dir

from hf_helpers import hf_model, our_last_logits

IDS = [5, 17, 3, 99, 42, 7, 250]


def _save(cfg, path, seed=0):
    torch.manual_seed(seed)
    m = hf_model(cfg)
    m.save_pretrained(str(path), safe_serialization=True)
    return m


def _hf_greedy(m, ids, max_length):
    with torch.no_grad():
        out = m.generate(torch.tensor([ids]), max_length=max_length, do_sample=False,
                         pad_token_id=0)
    return out[0].tolist()


@pytest.mark.parametrize("model", ["llama-tiny", "mixtral-tiny", "gpt2-tiny"])
def test_load_hf_dir_matches_hf_logits(tmp_path, model):
    cfg = get_config(model)
    m = _save(cfg, tmp_path / "ck")
    c2, params = load_hf_dir(tmp_path / "ck", dtype=torch.float32)
    assert (c2.hidden_size, c2.num_layers, c2.num_kv_heads, c2.num_experts, c2.arch) == (
        cfg.hidden_size, cfg.num_layers, cfg.num_kv_heads, cfg.num_experts, cfg.arch)
    with torch.no_grad():
        ref = m(torch.tensor([IDS])).logits[0, -1]
    ours = our_last_logits(c2, params, IDS)
    assert torch.allclose(ours, ref, atol=2e-4, rtol=1e-3), (ours - ref).abs().max()


def test_config_from_hf_real_shapes():
    c = config_from_hf({"model_type": "llama", "hidden_size": 4096, "num_attention_heads": 32,
                        "num_key_value_heads": 8, "num_hidden_layers": 32,
                        "intermediate_size": 14336, "vocab_size": 128256,
                        "rope_theta": 500000.0, "max_position_embeddings": 8192,
                        "bos_token_id": 128000, "eos_token_id": [128001, 128009]}, "x")
    ref = get_config("llama3-8b")
    assert (c.head_dim, c.num_kv_heads, c.rope_theta, c.eos_token_id) == (
        ref.head_dim, ref.num_kv_heads, ref.rope_theta, 128001)
    assert c.param_count() == ref.param_count()


def _worker(tmp_path):
    from distributed_llm_inferencing_amd.worker.server import create_worker_app
    s = Settings()
    s.master_db = str(tmp_path / "db.sqlite3")
    s.model_cache_dir = str(tmp_path / "cache")
    return create_worker_app(s, device="cpu", engine_kwargs=dict(max_batch=8, max_model_len=128,
                                                                 num_blocks=64))


@pytest.mark.parametrize("model,layout", [("llama-tiny", "plain"), ("mixtral-tiny", "hub"),
                                          ("gpt2-tiny", "plain")])
def test_worker_load_model_reads_hf_checkpoint(tmp_path, model, layout):
    cfg = get_config(model)
    name = f"acme/tiny-{model}"
    if layout == "plain":
        d = tmp_path / "cache" / name.replace("/", "_")
    else:
        hub = tmp_path / "cache" / ("models--" + name.replace("/", "--"))
        d = hub / "snapshots" / "0123abc"
        (hub / "refs").mkdir(parents=True)
        (hub / "refs" / "main").write_text("0123abc")
    m = _save(cfg, d, seed=3)
    assert find_hf_dir(str(tmp_path / "cache"), name) == d
    app = _worker(tmp_path)
    st = app.extensions["dli_worker"]
    c = app.test_client()
    r = c.post("/load_model", json={"model_name": name})
    assert r.status_code == 200, r.get_json()
    assert st.weights_source[name] == "cache"
    svc = st.services[name]
    from distributed_llm_inferencing_amd.engine import SamplingParams
    out = svc.generate(IDS, SamplingParams(max_length=24, do_sample=False, ignore_eos=True),
                       timeout=120)
    assert out.all_ids == _hf_greedy(m, IDS, 24)
    # the public route answers from the same weights
    r = c.post("/inference", json={"model_name": name, "prompt": "hi", "max_length": 12,
                                   "temperature": 0})
    assert r.status_code == 200 and r.get_json()["status"] == "success"
    st.unload_model(name)


def test_shard_model_from_hf_then_sharded_inference(tmp_path):
    from distributed_llm_inferencing_amd.shard.writer import main as shard_main
    cfg = get_config("llama-tiny")
    m = _save(cfg, tmp_path / "hf", seed=5)
    shard_main(["--model_name", "acme/llama", "--num_shards", "2", "--output_dir",
                str(tmp_path / "shards"), "--from-hf", str(tmp_path / "hf")])
    root = tmp_path / "shards" / "acme_llama"
    meta = [json.loads((root / f"shard_{i}" / "metadata.json").read_text()) for i in range(2)]
    assert [(x["start_layer"], x["end_layer"]) for x in meta] == [(0, 1), (2, 3)]
    app = _worker(tmp_path)
    c = app.test_client()
    for i in range(2):
        r = c.post("/load_shard", json={"model_name": "acme/llama", "shard_id": i,
                                        "shard_path": str(root / f"shard_{i}")})
        assert r.status_code == 200, r.get_json()
    st = app.extensions["dli_worker"]
    svc = st.shard_pipeline("acme/llama", [0, 1])
    from distributed_llm_inferencing_amd.engine import SamplingParams
    out = svc.generate(IDS, SamplingParams(max_length=20, do_sample=False, ignore_eos=True),
                       timeout=120)
    # shards are bf16 (the export dtype); compare against the HF model in bf16 as well
    assert len(out.all_ids) == 20 and out.all_ids[:len(IDS)] == IDS
    hb = _hf_greedy(m.to(torch.bfloat16), IDS, 20)
    agree = sum(a == b for a, b in zip(out.all_ids, hb))
    assert agree >= 16, (out.all_ids, hb)


@pytest.mark.parametrize("scaling", [
    {"rope_type": "llama3", "factor": 8.0, "low_freq_factor": 1.0, "high_freq_factor": 4.0,
     "original_max_position_embeddings": 16},
    {"rope_type": "linear", "factor": 4.0}])
def test_rope_scaling_matches_hf(tmp_path, scaling):
    """A Llama-3.1-style ``rope_scaling`` (llama3: long wavelengths divided by the factor,
    the band between smoothed; linear) changes every attention score past the first
    positions; it is absorbed into our cos/sin table and must give HF's logits. The same
    checkpoint read WITHOUT the scaling must not (the test has teeth)."""
    import dataclasses
    import transformers as tf
    cfg = get_config("llama-tiny")
    kw = dict(vocab_size=cfg.vocab_size, hidden_size=cfg.hidden_size,
              intermediate_size=cfg.intermediate_size, num_hidden_layers=cfg.num_layers,
              num_attention_heads=cfg.num_heads, num_key_value_heads=cfg.num_kv_heads,
              head_dim=cfg.head_dim, rms_norm_eps=cfg.norm_eps, max_position_embeddings=256,
              bos_token_id=1, eos_token_id=2, tie_word_embeddings=False)
    c = tf.LlamaConfig(rope_scaling=dict(scaling, rope_theta=10000.0), rope_theta=10000.0, **kw)
    torch.manual_seed(4)
    m = tf.LlamaForCausalLM(c).float().eval()
    m.save_pretrained(str(tmp_path / "ck"), safe_serialization=True)
    c2, params = load_hf_dir(tmp_path / "ck", dtype=torch.float32)
    assert dict(c2.rope_scaling).get("factor") == scaling["factor"]
    ids = [(7 * i + 3) % cfg.vocab_size for i in range(60)]
    with torch.no_grad():
        ref = m(torch.tensor([ids])).logits[0, -1]
    ours = our_last_logits(c2, params, ids)
    assert torch.allclose(ours, ref, atol=2e-4, rtol=1e-3), (ours - ref).abs().max()
    plain = our_last_logits(dataclasses.replace(c2, rope_scaling=()), params, ids)
    assert not torch.allclose(plain, ref, atol=2e-4, rtol=1e-3)


def test_unsupported_rope_scaling_and_sliding_window():
    base = {"model_type": "mistral", "hidden_size": 64, "num_attention_heads": 4,
            "num_hidden_layers": 2, "intermediate_size": 128, "vocab_size": 100,
            "max_position_embeddings": 32768}
    with pytest.raises(ValueError, match="unsupported rope_scaling"):
        config_from_hf(dict(base, rope_scaling={"rope_type": "yarn", "factor": 4.0}), "x")
    c = config_from_hf(dict(base, sliding_window=4096), "x")
    assert c.max_position == 4096          # context capped at the window, not silently wrong
