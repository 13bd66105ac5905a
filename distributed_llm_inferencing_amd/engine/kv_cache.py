"""Paged KV cache storage for one pipeline stage (its layers only).

Two tensors per stage (one allocation each, sized from free HBM):
    K: [L_stage, num_blocks, Hkv, block_size, hd]
    V: [L_stage, num_blocks, Hkv, block_size, hd]   (token-major like K, see ops/reference.py)
Zero-initialised once so rows past a sequence's context are always finite (the decode
kernel reads whole 32-token tiles and multiplies the masked ones by 0).
"""
from __future__ import annotations

from typing import List, Tuple

import torch

from ..models.configs import ModelConfig


def bytes_per_block(cfg: ModelConfig, num_layers: int, block_size: int, dtype_bytes: int = 2):
    return 2 * num_layers * cfg.num_kv_heads * cfg.head_dim * block_size * dtype_bytes


def blocks_for_budget(cfg: ModelConfig, num_layers: int, block_size: int, budget_bytes: int):
    return max(1, int(budget_bytes // max(1, bytes_per_block(cfg, num_layers, block_size))))


def auto_num_blocks(cfg: ModelConfig, num_layers: int, block_size: int, device,
                    fraction: float = 0.85, reserve_bytes: int = 4 << 30,
                    cap_tokens: int = 0) -> int:
    """Blocks that fit in `fraction` of currently free HBM minus a reserve for activations."""
    dev = torch.device(device)
    if dev.type == "cuda":
        free, _total = torch.cuda.mem_get_info(dev)
        budget = max(0, int(free * fraction) - reserve_bytes)
    else:
        budget = 256 << 20
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
