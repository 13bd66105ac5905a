"""Paged KV cache storage for one pipeline stage (its layers only).

Two tensors per stage (one allocation each, sized from free HBM):
    K: [L_stage, num_blocks, Hkv, block_size, hd]
    V: [L_stage, num_blocks, Hkv, block_size, hd]   (token-major like K, see ops/reference.py)
Zero-initialised once so rows past a sequence's context are always finite (the decode
kernel reads whole 32-token tiles and multiplies the masked ones by 0).
"""
from __future__ import annotations

import os
from typing import List, Optional, Tuple

import torch

from ..models.configs import ModelConfig


def bytes_per_block(cfg: ModelConfig, num_layers: int, block_size: int, dtype_bytes: int = 2):
    return 2 * num_layers * cfg.num_kv_heads * cfg.head_dim * block_size * dtype_bytes


def blocks_for_budget(cfg: ModelConfig, num_layers: int, block_size: int, budget_bytes: int):
    return max(1, int(budget_bytes // max(1, bytes_per_block(cfg, num_layers, block_size))))


def auto_num_blocks(cfg: ModelConfig, num_layers: int, block_size: int, device,
                    fraction: float = 0.85, reserve_bytes: Optional[int] = None,
                    cap_tokens: int = 0, pending_bytes: int = 0) -> int:
    """Blocks that fit in ``fraction`` of the HBM still free (weights already resident)
    minus a reserve for activations, GEMM workspaces and graph pools: the KV pool is sized
    for the 288 GB of an MI355X (Llama-3-8B: ~1.7M tokens of context on one GPU), not for
    max_batch x max_model_len. ``cap_tokens`` / ``DLI_KV_MAX_TOKENS`` cap it (0 = no cap).
    ``pending_bytes``: weights that will land on this device after the pool is sized (a
    pipeline stage sizes its pool before it loads its layers; ranks sharing one device pass
    every rank's). Ranks sharing one device (``DLI_SAME_DEVICE=1`` rehearsals) split the rest
    by ``LOCAL_WORLD_SIZE``."""
    dev = torch.device(device)
    env_cap = int(os.environ.get("DLI_KV_MAX_TOKENS", "0") or 0)
    cap_tokens = env_cap or cap_tokens
    if dev.type == "cuda":
        free, total = torch.cuda.mem_get_info(dev)
        free = max(0, free - int(pending_bytes))
        if reserve_bytes is None:
            reserve_bytes = max(8 << 30, int(0.03 * total))
        if os.environ.get("DLI_SAME_DEVICE", "0") == "1":
            ranks = os.environ.get("LOCAL_WORLD_SIZE", os.environ.get("WORLD_SIZE"))
            if ranks is None:
                # a worker that joined a ring by init_method (no launcher environment)
                import torch.distributed as dist
                ranks = dist.get_world_size() if dist.is_initialized() else 1
            fraction /= max(1, int(ranks))
        budget = max(0, int(free * fraction) - reserve_bytes)
    else:
        budget = 256 << 20                  # CPU (tests / the gpt2 plumbing config)
        cap_tokens = cap_tokens or (1 << 16)
    n = blocks_for_budget(cfg, max(1, num_layers), block_size, budget)
    if cap_tokens:
        n = min(n, -(-cap_tokens // block_size))
    return max(n, 16)


class KVCache:
    def __init__(self, cfg: ModelConfig, num_layers: int, num_blocks: int, block_size: int,
                 device, dtype=torch.bfloat16):
        self.cfg = cfg
        self.num_layers = num_layers
        self.num_blocks = num_blocks
        self.block_size = block_size
        hkv, hd = cfg.num_kv_heads, cfg.head_dim
        self.k = torch.zeros(num_layers, num_blocks, hkv, block_size, hd, dtype=dtype, device=device)
        self.v = torch.zeros(num_layers, num_blocks, hkv, block_size, hd, dtype=dtype, device=device)

    def layers(self) -> List[Tuple[torch.Tensor, torch.Tensor]]:
        return [(self.k[i], self.v[i]) for i in range(self.num_layers)]

    @property
    def nbytes(self) -> int:
        return 2 * self.k.numel() * self.k.element_size()

    @property
    def capacity_tokens(self) -> int:
        return self.num_blocks * self.block_size
