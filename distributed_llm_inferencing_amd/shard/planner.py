"""Layer-contiguous pipeline partitioning (reference: master/dashboard/management/commands/
shard_model.py:55-66) sized for 288 GB of HBM3E per MI355X.

Policies:
  even      the reference rule: layers_per_shard = L // N, the last shard also takes L % N
            (32 layers / 3 shards -> 10, 10, 12), same metadata.json schema.
  hbm       balance resident BYTES per GPU (embedding counted on the first stage, final norm
            + LM head on the last) so the largest shard is as small as possible.
  balanced  balance per-step TIME for decode, which is HBM-bandwidth bound: every layer's
            weights are streamed each step, the LM head (1 GB for Llama-3) is streamed on the
            last stage, but the embedding is only gathered (B rows). Default for serving.

All policies return contiguous [start, end) ranges and are validated against the per-GPU
HBM capacity (weights + a KV reserve).
"""
from __future__ import annotations

from dataclasses import asdict, dataclass
from typing import List, Sequence, Tuple

from ..models.configs import ModelConfig

HBM_BYTES = 288 * (1 << 30)


@dataclass
class StagePlan:
    shard_id: int
    start_layer: int
    end_layer: int            # exclusive
    weight_bytes: int
    time_cost: float
    first: bool
    last: bool

    def to_metadata(self, model_name: str, num_shards: int, total_layers: int) -> dict:
        """metadata.json as written by the reference (end_layer INCLUSIVE there)."""
        return {"model_name": model_name, "shard_id": self.shard_id, "num_shards": num_shards,
                "start_layer": self.start_layer, "end_layer": self.end_layer - 1,
                "total_layers": total_layers,
                # extensions (ignored by the reference's readers)
                "weight_bytes": self.weight_bytes, "first": self.first, "last": self.last}


def even_split(num_layers: int, n: int) -> List[Tuple[int, int]]:
    if n <= 0 or n > num_layers:
        raise ValueError(f"cannot split {num_layers} layers into {n} shards")
    lps, rem = divmod(num_layers, n)
    out = []
    for i in range(n):
        s = i * lps
        e = s + lps + (rem if i == n - 1 else 0)
        out.append((s, e))
    return out


def _min_max_partition(costs: Sequence[float], n: int, head_extra: float,
                       tail_extra: float) -> List[Tuple[int, int]]:
    """Contiguous partition of `costs` into n non-empty parts minimising the max part cost,
    with fixed extras on the first and last part. O(n L^2) DP (L <= ~128)."""
    L = len(costs)
    pre = [0.0]
    for c in costs:
        pre.append(pre[-1] + c)
    INF = float("inf")
    # best[k][j]: min max-cost splitting first j layers into k parts
    best = [[INF] * (L + 1) for _ in range(n + 1)]
    arg = [[0] * (L + 1) for _ in range(n + 1)]
    best[0][0] = 0.0
    for k in range(1, n + 1):
        for j in range(k, L - (n - k) + 1):
            for i in range(k - 1, j):
                part = pre[j] - pre[i]
                if k == 1:
                    part += head_extra
                if k == n and j == L:
                    part += tail_extra
                v = max(best[k - 1][i], part)
                if v < best[k][j]:
                    best[k][j] = v
                    arg[k][j] = i
    out, j = [], L
    for k in range(n, 0, -1):
        i = arg[k][j]
        out.append((i, j))
        j = i
    return out[::-1]


def plan_stages(cfg: ModelConfig, num_stages: int, policy: str = "balanced",
                dtype_bytes: int = 2, hbm_bytes: int = HBM_BYTES,
                kv_reserve_frac: float = 0.1, head_on_all: bool = False) -> List[StagePlan]:
    """``head_on_all``: the LM head runs vocab-parallel on every stage (parallel/pipeline.py),
    so its cost is the same on each stage and the layers split evenly."""
    L = cfg.num_layers
    layer_b = cfg.layer_param_count() * dtype_bytes
    embed_b = cfg.embed_param_count() * dtype_bytes
    head_b = cfg.head_param_count() * dtype_bytes
    if policy == "even":
        ranges = even_split(L, num_stages)
    elif policy == "hbm":
        ranges = _min_max_partition([layer_b] * L, num_stages, embed_b, head_b)
    elif policy == "balanced":
        # decode step time ~ bytes streamed; the LM head is streamed, the embedding gathered;
        # the sampler over the vocab costs roughly one more pass over fp32 logits
        tail_time = 0 if head_on_all else head_b + 4 * cfg.vocab_size * 256
        ranges = _min_max_partition([float(layer_b)] * L, num_stages, 0.0, float(tail_time))
    else:
        raise ValueError(f"unknown policy {policy}")
    plans = []
    for i, (s, e) in enumerate(ranges):
        first, last = i == 0, i == len(ranges) - 1
        wb = (e - s) * layer_b + (embed_b if first else 0) + (head_b if last else 0)
        if last and cfg.tie_embeddings and not first:
            wb += embed_b
        if head_on_all:
            tc = (e - s) * layer_b + (head_b + 4 * cfg.vocab_size * 256) / len(ranges)
        else:
            tc = (e - s) * layer_b + ((head_b + 4 * cfg.vocab_size * 256) if last else 0)
        plans.append(StagePlan(i, s, e, wb, float(tc), first, last))
    limit = hbm_bytes * (1 - kv_reserve_frac)
    for p in plans:
        if p.weight_bytes > limit:
            raise ValueError(f"shard {p.shard_id} needs {p.weight_bytes / 2**30:.1f} GiB of "
                             f"weights > {limit / 2**30:.1f} GiB usable HBM; use more stages")
    return plans


def summarize(plans: List[StagePlan]) -> List[dict]:
    return [asdict(p) for p in plans]
