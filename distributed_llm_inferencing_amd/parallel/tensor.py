"""Tensor parallelism (optional, for ablation against the
layer-sharded pipeline — not the north star).

Megatron-style split of every Llama layer over N ranks:
    wqkv   column-parallel by heads (Hq/N query heads, Hkv/N kv heads per rank)
    wo     row-parallel (the rank's query-head columns) -> all-reduce(sum)
    w_gu   column-parallel in whole 32-row gate/up interleave groups (F/N features)
    w_down row-parallel -> all-reduce(sum)
Embedding, norms and the LM head are replicated; every rank samples the same token with
the same per-request Philox seed (deterministic kernels), so no logits gather is needed.
Each rank keeps the KV cache of its own Hkv/N heads. On an 8-GPU xGMI mesh the two
all-reduces per layer are per-link bound (ring over 7 links), which is why the pipeline is
the default for serving; this mode exists to measure that trade-off.
Ranks run identical schedulers on identical request streams (lockstep by construction).
"""
from __future__ import annotations

import os
import time
from dataclasses import replace
from typing import Optional

import torch
import torch.distributed as dist

from ..engine.llm_engine import LLMEngine
from ..models import weights as W
from ..models.configs import get_config
from ..models.model import TransformerLM
from ..ops.reference import GU_GROUP


def shard_param(name: str, t: torch.Tensor, cfg, rank: int, world: int) -> torch.Tensor:
    hd, hq, hkv = cfg.head_dim, cfg.num_heads, cfg.num_kv_heads
    if name.endswith(".wqkv"):
        q = t[: hq * hd].view(hq, hd, -1)
        k = t[hq * hd:(hq + hkv) * hd].view(hkv, hd, -1)
        v = t[(hq + hkv) * hd:].view(hkv, hd, -1)
        qs, ks = hq // world, hkv // world
        parts = [q[rank * qs:(rank + 1) * qs], k[rank * ks:(rank + 1) * ks],
                 v[rank * ks:(rank + 1) * ks]]
        return torch.cat([p.reshape(-1, t.shape[1]) for p in parts]).contiguous()
    if name.endswith(".wo"):
        qs = hq // world
        return t[:, rank * qs * hd:(rank + 1) * qs * hd].contiguous()
    if name.endswith(".w_gu"):
        rows = t.shape[0] // world
        return t[rank * rows:(rank + 1) * rows].contiguous()
    if name.endswith(".w_down"):
        cols = t.shape[1] // world
        return t[:, rank * cols:(rank + 1) * cols].contiguous()
    return t


class TPReduce:
    def __init__(self, group=None):
        self.group = group
        self.calls = 0

    def __call__(self, x: torch.Tensor) -> torch.Tensor:
        self.calls += 1
        if dist.get_backend(self.group) == "nccl" or not x.is_cuda:
            dist.all_reduce(x, group=self.group)
            return x
        y = x.float().cpu()
        dist.all_reduce(y, group=self.group)
        x.copy_(y.to(x.dtype))
        return x


class TensorParallelEngine:
    def __init__(self, model: str, device, max_batch: int = 256, max_model_len: int = 2048,
                 seed: int = 0, num_blocks: Optional[int] = None, dtype=torch.bfloat16,
                 max_prefill_tokens: int = 16384):
        from .transport import init_distributed
        dev = torch.device(device)
        self.rank, self.world = init_distributed(device=dev if dev.type == "cuda" else None)
        full = get_config(model)
        if full.is_moe or full.arch != "llama":
            raise ValueError("tensor parallel mode supports the dense Llama family")
        n = self.world
        if full.num_heads % n or full.num_kv_heads % n or full.intermediate_size % (GU_GROUP * n):
            raise ValueError(f"{model} does not split over {n} ranks")
        self.full_cfg = full
        local = replace(full, num_heads=full.num_heads // n, num_kv_heads=full.num_kv_heads // n,
                        intermediate_size=full.intermediate_size // n)
        shapes = W.stage_param_shapes(full, 0, full.num_layers, True, True)
        params = {}
        for name, shape in shapes.items():
            t = W.random_init({name: shape}, dev, dtype, seed)[name]
            params[name] = shard_param(name, t, full, self.rank, n)
            del t
        lm = TransformerLM(local, params, device=dev)
        self.reduce = TPReduce()
        lm.tp_reduce = self.reduce
        self.engine = LLMEngine(local, device=str(dev), dtype=dtype, max_batch=max_batch,
                                max_model_len=max_model_len, num_blocks=num_blocks,
                                use_graphs=False, lm=lm, max_prefill_tokens=max_prefill_tokens,
                                lookahead=False,   # lockstep all-reduces on every rank
                                mixed_steps=False)
        self.device = dev

    def generate(self, prompts, params=None):
        return self.engine.generate(prompts, params)


def bench_tensor_parallel(args, world, rank, make_prompts):
    local = int(os.environ.get("LOCAL_RANK", rank))
    if os.environ.get("DLI_SAME_DEVICE", "0") == "1":
        local = 0
    if torch.cuda.is_available():
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
    else:
        dev = torch.device("cpu")
    batch = args.batch * world          # per-GPU share of the weights shrinks, batch grows
    eng = TensorParallelEngine(args.model, dev, max_batch=batch,
                               max_model_len=args.max_model_len,
                               max_prefill_tokens=max(batch * args.prompt_len, 8192))
    from ..engine.sequence import SamplingParams
    sp = SamplingParams(max_length=args.max_length, temperature=0.8, top_k=50, top_p=0.95,
                        ignore_eos=True, seed=1234)

    def wave(seed):
        outs = eng.generate(make_prompts(batch, args.prompt_len, eng.full_cfg.vocab_size,
                                         seed), sp)
        return sum(len(o.output_ids) for o in outs), [o.latency_s for o in outs]

    for w in range(args.warmup):
        wave(10_000 + w)
    dist.barrier()
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    toks, lats = 0, []
    for s in range(args.steps):
        n, l = wave(s)
        toks += n
        lats += l
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    dist.barrier()
    cdev = dev if dist.get_backend() == "nccl" else torch.device("cpu")
    dt = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=cdev)
    dist.all_reduce(dt, op=dist.ReduceOp.MAX)
    from .transport import gather_rank_info
    infos = gather_rank_info(dev)
    dist.barrier()
    plane = "torch-rccl" if dist.get_backend() == "nccl" else "torch-gloo"
    dist.destroy_process_group()
    if rank != 0:
        return None
    # every rank produced the same tokens for the same requests: count them once
    return {"tokens": toks, "seconds": float(dt.item()), "latencies": lats,
            "global_batch": batch, "parallelism": f"tp{world}", "data_plane": plane,
            "ranks_info": infos}
