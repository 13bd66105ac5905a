"""Expert parallelism for Mixtral: experts mapped to GPU ranks, all-to-all over xGMI
(BASELINE.json config 5; SURVEY.md §2.4 C4, §2.5 "Expert parallel").

Layout: data-parallel attention + expert-parallel MoE. Every rank holds the full attention
/ norm / embedding weights and its own requests + paged KV; rank r holds experts
[r*E/N, (r+1)*E/N). Per MoE layer:

    route (softmax -> top-2 -> renormalise, local)
    dispatch: (token, slot) rows sorted by destination rank -> all_to_all_single
    local grouped-GEMM expert MLPs (HIP kernels) on the rows received
    combine: all_to_all_single back -> weighted sum per token

On the fully connected 8-GPU xGMI mesh each rank pair has its own link, so the all-to-all
runs on all 7 links at once. Split sizes are exchanged per layer (one tiny all-to-all of
counts) so the payload is exact (no capacity padding / no dropped tokens).

Ranks step in lockstep (each step runs the same 32 MoE exchanges on every rank; a rank with
no local work still joins with zero rows).
"""
from __future__ import annotations

import os
import time
from typing import Optional

import torch
import torch.distributed as dist

from .. import ops
from ..engine.llm_engine import LLMEngine
from ..models.configs import get_config
from ..models.model import TransformerLM
from ..models import weights as W


class ExpertParallelMoE:
    """Installed as ``TransformerLM.moe_fn`` on every rank."""

    def __init__(self, num_experts: int, top_k: int, group=None):
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        if num_experts % self.world:
            raise ValueError(f"{num_experts} experts do not split over {self.world} ranks")
        self.E, self.k = num_experts, top_k
        self.e_per = num_experts // self.world
        self.e0 = self.rank * self.e_per
        self.bytes_sent = 0
        self.exchanges = 0

    def expert_range(self):
        return (self.e0, self.e0 + self.e_per)

    def _a2a(self, out, inp, out_splits, in_splits):
        dist.all_to_all_single(out, inp, out_splits, in_splits, group=self.group)

    def __call__(self, h: torch.Tensor, lp: dict, layer: int) -> torch.Tensor:
        T, D = h.shape
        dev = h.device
        k, N = self.k, self.world
        if T > 0:
            router_logits = ops.linear(h, lp["router"])
            topk_w, topk_ids = ops.moe_route(router_logits, k)
            flat_ids = topk_ids.reshape(-1).long()
            dest = flat_ids // self.e_per
            order = torch.argsort(dest, stable=True)
            send_counts = torch.bincount(dest, minlength=N)
        else:
            topk_w = torch.zeros(0, k, dtype=torch.float32, device=dev)
            flat_ids = torch.zeros(0, dtype=torch.long, device=dev)
            order = torch.zeros(0, dtype=torch.long, device=dev)
            send_counts = torch.zeros(N, dtype=torch.long, device=dev)
        cdev = dev if dist.get_backend(self.group) == "nccl" else torch.device("cpu")
        sc = send_counts.to(cdev)
        rc = torch.empty_like(sc)
        dist.all_to_all_single(rc, sc, group=self.group)
        in_splits = sc.tolist()
        out_splits = rc.tolist()
        R = int(sum(out_splits))
        # dispatch rows (token embedding + its global expert id)
        src_tok = order // k
        send_x = h.index_select(0, src_tok) if T > 0 else h.new_zeros(0, D)
        send_e = flat_ids.index_select(0, order).to(torch.int32) if T > 0 else \
            torch.zeros(0, dtype=torch.int32, device=dev)
        recv_x = torch.empty(R, D, dtype=h.dtype, device=cdev)
        recv_e = torch.empty(R, dtype=torch.int32, device=cdev)
        self._a2a(recv_x, send_x.to(cdev), out_splits, in_splits)
        self._a2a(recv_e, send_e.to(cdev), out_splits, in_splits)
        recv_x, recv_e = recv_x.to(dev), recv_e.to(dev)
        # local experts: one expert per received row (top-1 with weight 1)
        if R > 0:
            y = ops.moe_mlp(recv_x, lp["w_gu"], lp["w_down"],
                            torch.ones(R, 1, dtype=torch.float32, device=dev),
                            recv_e.view(R, 1), self.e0)
        else:
            y = recv_x.new_zeros(0, D)
        back = torch.empty(T * k, D, dtype=h.dtype, device=cdev)
        self._a2a(back, y.to(cdev), in_splits, out_splits)
        back = back.to(dev)
        self.exchanges += 1
        self.bytes_sent += (T * k + R) * D * h.element_size()
        if T == 0:
            return h.new_zeros(0, D)
        contrib = torch.empty_like(back)
        contrib.index_copy_(0, order, back)
        out = (contrib.view(T, k, D).float() * topk_w.view(T, k, 1)).sum(1)
        return out.to(h.dtype)


class ExpertParallelEngine:
    """One rank of a DP-attention / EP-MoE Mixtral deployment (all ranks are peers; each
    serves its own requests)."""

    def __init__(self, model: str, device, max_batch: int = 256, max_model_len: int = 2048,
                 seed: int = 0, num_blocks: Optional[int] = None, dtype=torch.bfloat16,
                 max_prefill_tokens: int = 16384):
        from .transport import init_distributed
        dev = torch.device(device)
        self.rank, self.world = init_distributed(device=dev if dev.type == "cuda" else None)
        cfg = get_config(model)
        if not cfg.is_moe:
            raise ValueError(f"{model} has no experts")
        self.cfg = cfg
        self.moe = ExpertParallelMoE(cfg.num_experts, cfg.top_k_experts)
        er = self.moe.expert_range()
        shapes = W.stage_param_shapes(cfg, 0, cfg.num_layers, True, True)
        params = {}
        # generate full tensors per name (deterministic) and keep only the local experts
        for name, shape in shapes.items():
            t = W.random_init({name: shape}, dev, dtype, seed)[name]
            params[name] = W.slice_experts(name, t, er)
            del t
        lm = TransformerLM(cfg, params, device=dev, expert_range=er)
        lm.moe_fn = self.moe
        self.engine = LLMEngine(cfg, device=str(dev), dtype=dtype, max_batch=max_batch,
                                max_model_len=max_model_len, num_blocks=num_blocks,
                                use_graphs=False, lm=lm,
                                max_prefill_tokens=max_prefill_tokens,
                                lookahead=False)   # every forward joins the ranks' all-to-alls
        self.device = dev

    def _any_work(self) -> bool:
        cdev = self.device if dist.get_backend() == "nccl" else torch.device("cpu")
        t = torch.tensor([1 if self.engine.has_work() else 0], dtype=torch.int32, device=cdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return bool(t.item())

    def _idle_step(self):
        """Join every MoE exchange of one forward with zero local rows."""
        D = self.cfg.hidden_size
        h = torch.zeros(0, D, dtype=torch.bfloat16, device=self.device)
        for i in range(self.cfg.num_layers):
            self.moe(h, self.engine.model.layers[i], i)

    def run_until_idle(self):
        outs = []
        while self._any_work():
            if self.engine.has_work():
                outs.extend(self.engine.step())
            else:
                self._idle_step()
        outs.extend(self.engine.step())
        return outs

    def generate(self, prompts, params=None):
        rids = [self.engine.add_request(p, params) for p in prompts]
        done = {o.request_id: o for o in self.run_until_idle()}
        return [done[r] for r in rids]


def bench_expert_parallel(args, world, rank, make_prompts):
    local = int(os.environ.get("LOCAL_RANK", rank))
    if os.environ.get("DLI_SAME_DEVICE", "0") == "1":
        local = 0
    if torch.cuda.is_available():
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
    else:
        dev = torch.device("cpu")
    eng = ExpertParallelEngine(args.model, dev, max_batch=args.batch,
                               max_model_len=args.max_model_len,
                               max_prefill_tokens=max(args.batch * args.prompt_len, 8192))
    from ..engine.sequence import SamplingParams
    sp = SamplingParams(max_length=args.max_length, temperature=0.8, top_k=50, top_p=0.95,
                        ignore_eos=True)

    def wave(seed):
        outs = eng.generate(make_prompts(args.batch, args.prompt_len, eng.cfg.vocab_size,
                                         seed * 100 + rank), sp)
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
    tt = torch.tensor([toks], dtype=torch.float64, device=cdev)
    dist.all_reduce(tt)
    lat_t = torch.tensor(lats, dtype=torch.float64, device=cdev)
    gathered = [torch.zeros_like(lat_t) for _ in range(world)]
    dist.all_gather(gathered, lat_t)
    dist.barrier()
    dist.destroy_process_group()
    if rank != 0:
        return None
    return {"tokens": int(tt.item()), "seconds": float(dt.item()),
            "latencies": torch.cat(gathered).tolist(), "global_batch": args.batch * world,
            "parallelism": f"dp{world}-ep{world}"}
