"""Builders for HF transformers twins of our tiny configs (the reference's runtime)."""
import numpy as np
import torch

from distributed_llm_inferencing_amd.engine.batch import PREFILL, StepMeta, to_device
from distributed_llm_inferencing_amd.models import TransformerLM
from distributed_llm_inferencing_amd.models.weights import from_hf_state_dict


def hf_model(cfg):
    import transformers as tf
    if cfg.arch == "gpt2":
        c = tf.GPT2Config(vocab_size=cfg.vocab_size, n_positions=cfg.max_position,
                          n_embd=cfg.hidden_size, n_layer=cfg.num_layers, n_head=cfg.num_heads,
                          n_inner=cfg.intermediate_size, bos_token_id=cfg.bos_token_id,
                          eos_token_id=cfg.eos_token_id)
        return tf.GPT2LMHeadModel(c).float().eval()
    kw = dict(vocab_size=cfg.vocab_size, hidden_size=cfg.hidden_size,
              intermediate_size=cfg.intermediate_size, num_hidden_layers=cfg.num_layers,
              num_attention_heads=cfg.num_heads, num_key_value_heads=cfg.num_kv_heads,
              head_dim=cfg.head_dim, rope_theta=cfg.rope_theta, rms_norm_eps=cfg.norm_eps,
              max_position_embeddings=cfg.max_position, bos_token_id=cfg.bos_token_id,
              eos_token_id=cfg.eos_token_id, tie_word_embeddings=False)
    if cfg.is_moe:
        c = tf.MixtralConfig(num_local_experts=cfg.num_experts,
                             num_experts_per_tok=cfg.top_k_experts, **kw)
        return tf.MixtralForCausalLM(c).float().eval()
    return tf.LlamaForCausalLM(tf.LlamaConfig(**kw)).float().eval()


def prefill_meta(ids):
    T = len(ids)
    return StepMeta(kind=PREFILL, seq_ids=[0], input_ids=np.array(ids, np.int32),
                    positions=np.arange(T, dtype=np.int32), slot_mapping=-np.ones(T, np.int32),
                    seq_lens=np.array([T], np.int32), context_lens=np.array([T], np.int32),
                    block_tables=np.zeros((1, 0), np.int32),
                    temperature=np.zeros(1, np.float32), top_k=np.ones(1, np.int32),
                    top_p=np.ones(1, np.float32), seeds=np.zeros(1, np.int64))


def our_last_logits(cfg, params, ids, device="cpu"):
    m = TransformerLM(cfg, params, device=device)
    db = to_device(prefill_meta(ids), device)
    x = m.forward_layers(m.embed(db), db, [])
    return m.logits(x, db)[0]
