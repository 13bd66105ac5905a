#!/usr/bin/env python3
"""The reference's execution strategy measured on MI355X (SURVEY.md §6 / BASELINE.md):
HF transformers AutoModelForCausalLM.generate, batch 1, requests served one at a time
(1 sync gunicorn worker, worker/Dockerfile:45), do_sample T=0.8 top_k=50 top_p=0.95,
max_length=100 including a 32-token synthetic prompt, random-init weights, bf16 on GPU.
Writes profiles/reference_strategy.json (bench.py divides by it for vs_baseline).

``--batch B`` runs the same HF ``generate`` on B prompts at once instead (not the
reference's strategy: a like-for-like comparator for bench.py's batch-512 wave).""" 
import argparse
import json
import statistics
import time
from pathlib import Path

import numpy as np
import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--requests", type=int, default=6)
    ap.add_argument("--prompt-len", type=int, default=32)
    ap.add_argument("--max-length", type=int, default=100)
    ap.add_argument("--out", default="profiles/reference_strategy.json")
    ap.add_argument("--batch", type=int, default=1,
                    help="prompts per generate call (1 = the reference's strategy)")
    a = ap.parse_args()
    import sys
    sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
    import transformers as tf
    from distributed_llm_inferencing_amd.models import get_config
    cfg = get_config(a.model)
    hc = tf.LlamaConfig(vocab_size=cfg.vocab_size, hidden_size=cfg.hidden_size,
                        intermediate_size=cfg.intermediate_size, num_hidden_layers=cfg.num_layers,
                        num_attention_heads=cfg.num_heads, num_key_value_heads=cfg.num_kv_heads,
                        head_dim=cfg.head_dim, rope_theta=cfg.rope_theta,
                        max_position_embeddings=cfg.max_position, bos_token_id=cfg.bos_token_id,
                        eos_token_id=cfg.eos_token_id)
    torch.set_default_dtype(torch.bfloat16)
    with torch.device("cuda"):
        model = tf.LlamaForCausalLM(hc).eval()
    rng = np.random.default_rng(0)
    lats, toks = [], 0
    for r in range(a.requests + 1):
        ids = torch.tensor([rng.integers(1000, cfg.vocab_size - 1000, a.prompt_len).tolist()
                            for _ in range(a.batch)], device="cuda")
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with torch.no_grad():
            out = model.generate(ids, max_length=a.max_length, num_return_sequences=1,
                                 do_sample=True, top_p=0.95, top_k=50, temperature=0.8,
                                 eos_token_id=None, pad_token_id=0)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        if r == 0:
            continue  # warmup
        lats.append(dt)
        toks += a.batch * (out.shape[1] - a.prompt_len)
    res = {"metric": ("output tokens/sec (reference strategy: HF generate, batch 1, serial)"
                      if a.batch == 1 else
                      f"output tokens/sec (HF generate, {a.batch} prompts per call)"),
           "batch": a.batch,
           "value": toks / sum(lats), "p50_latency_s": statistics.median(lats),
           "requests": a.requests, "model": a.model, "transformers": tf.__version__,
           "torch": torch.__version__, "device": torch.cuda.get_device_name(0)}
    Path(a.out).parent.mkdir(parents=True, exist_ok=True)
    Path(a.out).write_text(json.dumps(res, indent=2))
    print(json.dumps(res))


if __name__ == "__main__":
    main()
