"""Our model definitions vs HF transformers (the runtime the reference worker calls,
worker/app.py:121,297) on shared random weights: logits parity and greedy-generation parity."""
import pytest
import torch

from distributed_llm_inferencing_amd.engine import SamplingParams
from distributed_llm_inferencing_amd.engine.llm_engine import LLMEngine
from distributed_llm_inferencing_amd.models import get_config
from distributed_llm_inferencing_amd.models.weights import from_hf_state_dict

from hf_helpers import hf_model, our_last_logits

IDS = [5, 17, 99, 3, 250, 7, 8, 1000, 42, 11]


@pytest.mark.parametrize("name", ["llama-tiny", "gpt2-tiny", "mixtral-tiny", "llama-tiny128"])
def test_logits_match_hf_fp32(name):
    torch.manual_seed(0)
    cfg = get_config(name)
    hm = hf_model(cfg)
    with torch.no_grad():
        ref = hm(torch.tensor([IDS])).logits[0, -1]
    ours = our_last_logits(cfg, from_hf_state_dict(cfg, hm.state_dict(), dtype=torch.float32), IDS)
    assert torch.allclose(ours, ref, atol=2e-5, rtol=1e-4), (ours - ref).abs().max()


@pytest.mark.parametrize("name", ["llama-tiny", "gpt2-tiny", "mixtral-tiny"])
def test_greedy_generation_matches_hf_generate(name):
    """Paged-KV decode loop == HF generate(do_sample=False) token for token (fp32)."""
    torch.manual_seed(1)
    cfg = get_config(name)
    hm = hf_model(cfg)
    params = from_hf_state_dict(cfg, hm.state_dict(), dtype=torch.float32)
    eng = LLMEngine(cfg, device="cpu", dtype=torch.float32, params=params, max_batch=4,
                    max_model_len=64, num_blocks=32, block_size=16)
    prompts = [IDS[:6], IDS[2:9], IDS[:3]]
    outs = eng.generate(prompts, SamplingParams(max_length=20, do_sample=False, ignore_eos=True))
    for p, o in zip(prompts, outs):
        with torch.no_grad():
            ref = hm.generate(torch.tensor([p]), max_length=20, do_sample=False,
                              eos_token_id=None, pad_token_id=0)[0].tolist()
        assert o.all_ids == ref, (o.all_ids, ref)
