#!/usr/bin/env python3
"""BASELINE config 1: gpt2 on one CPU worker. Reference strategy (HF generate, batch 1,
serial) vs this framework's CPU engine (continuous batching over the PyTorch reference ops).
Random-init GPT-2 (124M) weights shared by both; 32-token prompts, max_length 100."""
import json
import statistics
import sys
import time
from pathlib import Path

import numpy as np
import torch

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from distributed_llm_inferencing_amd.engine import SamplingParams  # noqa: E402
from distributed_llm_inferencing_amd.engine.llm_engine import LLMEngine  # noqa: E402
from distributed_llm_inferencing_amd.models import get_config  # noqa: E402
from distributed_llm_inferencing_amd.models.weights import from_hf_state_dict  # noqa: E402


def main(n_ref=3, n_ours=16):
    import transformers as tf
    cfg = get_config("gpt2")
    torch.manual_seed(0)
    hm = tf.GPT2LMHeadModel(tf.GPT2Config()).eval()
    rng = np.random.default_rng(0)
    prompts = [rng.integers(100, 50000, 32).tolist() for _ in range(max(n_ref, n_ours))]
    lat = []
    for p in prompts[:n_ref]:
        t0 = time.perf_counter()
        with torch.no_grad():
            hm.generate(torch.tensor([p]), max_length=100, do_sample=True, top_p=0.95, top_k=50,
                        temperature=0.8, eos_token_id=None, pad_token_id=0)
        lat.append(time.perf_counter() - t0)
    ref = {"tok_s": 68 * n_ref / sum(lat), "p50_s": statistics.median(lat)}
    params = from_hf_state_dict(cfg, hm.state_dict(), dtype=torch.float32)
    eng = LLMEngine(cfg, device="cpu", dtype=torch.float32, params=params, max_batch=n_ours,
                    max_model_len=128, num_blocks=16 * n_ours)
    sp = SamplingParams(max_length=100, ignore_eos=True)
    t0 = time.perf_counter()
    outs = eng.generate(prompts[:n_ours], sp)
    dt = time.perf_counter() - t0
    ours = {"tok_s": sum(len(o.output_ids) for o in outs) / dt,
            "p50_s": statistics.median(o.latency_s for o in outs), "concurrent": n_ours}
    # same serial batch-1 strategy as the reference, for a like-for-like latency
    lat1 = [eng.generate([p], sp)[0].latency_s for p in prompts[:n_ref]]
    ours_b1 = {"tok_s": 68 * n_ref / sum(lat1), "p50_s": statistics.median(lat1)}
    res = {"config": "gpt2, 1 CPU worker", "reference_strategy": ref, "ours": ours,
           "ours_batch1_serial": ours_b1,
           "threads": torch.get_num_threads()}
    print(json.dumps(res))
    Path("profiles").mkdir(exist_ok=True)
    Path("profiles/cpu_gpt2.json").write_text(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
