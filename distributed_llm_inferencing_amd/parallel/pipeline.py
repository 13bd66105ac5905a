"""Layer-sharded pipeline-parallel serving: one process per MI355X, stages over RCCL.

This is what the reference's "sharded inference" was meant to be (offline
layer split, ``metadata.json``, ``/load_shard``; execution never actually coordinated the
shards) — made real:

* stage r holds layers [start_r, end_r) (shard/planner.py), its own paged KV pool and its
  own hipGraph-captured decode step;
* rank 0 (the head) owns the scheduler, the C++ block allocator and the tokenizer; every
  step's packed metadata rides with the activations through the ring, so the other stages
  hold no scheduling state at all;
* M = N microbatches circulate: while microbatch m is in stage r, stage r-1 runs m+1, so
  all N GPUs are busy in steady state; the tail samples on device and returns int32 tokens
  to the head (C3), which schedules that microbatch's next step one ring later;
* sessions: the head drives the ring while it has work, then sends STOP; other ranks
  block waiting for the next session; SHUTDOWN ends them.

``LocalPipeline`` runs the same partitioned stages and tick schedule in ONE process (all
stages on one device): the loopback transport used to test pipeline correctness on a single
GPU or CPU.
"""
from __future__ import annotations

import os
import time
from typing import Dict, List, Optional

import numpy as np
import torch
import torch.distributed as dist

from ..engine.batch import DECODE, EMPTY, HEADER_LEN, PREFILL, STOP, StepMeta
from ..engine.kv_cache import KVCache, auto_num_blocks
from ..engine.llm_engine import EngineStats, seq_to_output
from ..engine.runner import StageRunner
from ..engine.scheduler import Scheduler
from ..engine.sequence import RequestOutput, SamplingParams
from ..models.configs import ModelConfig, get_config
from ..models.model import TransformerLM
from ..runtime import BlockManager
from ..shard.planner import StagePlan, plan_stages
from ..tokenizer import load_tokenizer
from .transport import (DATA_HIDDEN, DATA_NONE, DATA_TOKENS, H_DATA_COLS, H_DATA_KIND,
                        H_DATA_ROWS, H_TICK, Message, TorchDistTransport, init_distributed)

SHUTDOWN = 4


def _control(kind: int, tick: int) -> Message:
    h = np.zeros(HEADER_LEN, dtype=np.int64)
    h[0] = kind
    h[H_TICK] = tick
    return Message(header=h, payload=np.zeros(0, dtype=np.int32), data=None)


def _msg_from(meta: StepMeta, data: Optional[torch.Tensor], tick: int, tokens: bool) -> Message:
    h, payload = meta.pack()
    h[H_TICK] = tick
    if data is None:
        h[H_DATA_KIND] = DATA_NONE
    elif tokens:
        h[H_DATA_KIND], h[H_DATA_ROWS] = DATA_TOKENS, data.shape[0]
    else:
        h[H_DATA_KIND], h[H_DATA_ROWS], h[H_DATA_COLS] = DATA_HIDDEN, data.shape[0], data.shape[1]
    return Message(header=h, payload=payload, data=data)


class StageWorker:
    """Model slice + KV pool + hipGraph runner of one pipeline stage."""

    def __init__(self, cfg: ModelConfig, plan: StagePlan, device, num_blocks: int,
                 block_size: int, max_batch: int, table_width: int, seed: int = 0,
                 use_graphs: Optional[bool] = None, params=None, dtype=torch.bfloat16):
        self.cfg, self.plan = cfg, plan
        self.device = torch.device(device)
        if params is None:
            self.model = TransformerLM.random(cfg, plan.start_layer, plan.end_layer, self.device,
                                              dtype=dtype, seed=seed)
        else:
            self.model = TransformerLM(cfg, {k: v.to(self.device) for k, v in params.items()},
                                       plan.start_layer, plan.end_layer, self.device)
        self.kv = KVCache(cfg, plan.end_layer - plan.start_layer, num_blocks, block_size,
                          self.device, dtype)
        self.runner = StageRunner(self.model, self.kv, max_batch, table_width, use_graphs)

    @property
    def is_last(self) -> bool:
        return self.model.is_last

    def compute(self, meta: StepMeta, data: Optional[torch.Tensor]) -> Optional[torch.Tensor]:
        if meta.kind not in (PREFILL, DECODE) or meta.num_seqs == 0:
            return None
        return self.runner.run(meta, hidden=data)


def _stage_capacity_blocks(cfg, plan, block_size, device, kv_fraction, cap_tokens):
    return auto_num_blocks(cfg, plan.end_layer - plan.start_layer, block_size, device,
                           kv_fraction, cap_tokens=cap_tokens)


class PipelineHead:
    """Rank-0 driver: scheduler + ring ticks (M = N microbatches)."""

    def __init__(self, stage: StageWorker, transport, scheduler: Scheduler, tokenizer):
        self.stage, self.tp, self.sched, self.tok = stage, transport, scheduler, tokenizer
        self.N = transport.world
        self.stats = EngineStats()

    def run_session(self) -> List[RequestOutput]:
        N, k = self.N, 0
        inflight: Dict[int, Optional[StepMeta]] = {}
        results: Dict[int, np.ndarray] = {}
        while True:
            j = k - N
            if j >= 0:
                m = inflight.pop(j, None)
                if m is not None:
                    self.sched.update(m, results.pop(j))
                    self.stats.tokens_out += m.num_seqs
                else:
                    results.pop(j, None)
            live = any(v is not None for v in inflight.values())
            meta = self.sched.schedule(k % N) if self.sched.has_work() else None
            if meta is None and not live and not self.sched.has_work():
                self.tp.exchange(_control(STOP, k), recv=(k - N + 1) >= 0)
                break
            t0 = time.perf_counter()
            if meta is None:
                msg = _control(EMPTY, k)
            else:
                hidden = self.stage.compute(meta, None)
                msg = _msg_from(meta, hidden, k, tokens=False)
                self.stats.steps += 1
                if meta.kind == PREFILL:
                    self.stats.prefill_steps += 1
                    self.stats.prompt_tokens += meta.num_tokens
                else:
                    self.stats.decode_steps += 1
            inflight[k] = meta
            got = self.tp.exchange(msg, recv=(k - N + 1) >= 0)
            if got is not None:
                tick = int(got.header[H_TICK])
                results[tick] = (got.data.cpu().numpy() if got.data is not None
                                 else np.zeros(0, np.int32))
            self.stats.busy_s += time.perf_counter() - t0
            k += 1
        # drain the ring until our STOP comes back from the tail
        while True:
            got = self.tp.exchange(None, recv=True)
            if int(got.header[0]) == STOP:
                break
        outs = []
        for seq in self.sched.pop_finished():
            o = seq_to_output(seq, self.tok)
            self.stats.finished += 1
            self.stats.latencies.append(o.latency_s)
            outs.append(o)
        return outs

    def shutdown(self):
        self.tp.exchange(_control(SHUTDOWN, -1), recv=False)
        got = self.tp.exchange(None, recv=True)          # SHUTDOWN returns from the tail
        assert int(got.header[0]) == SHUTDOWN


def run_stage_loop(stage: StageWorker, transport) -> None:
    """Non-head ranks: serve sessions until SHUTDOWN."""
    while True:
        msg = transport.exchange(None, recv=True)
        while True:
            kind = int(msg.header[0])
            if kind in (STOP, SHUTDOWN):
                transport.exchange(_control(kind, int(msg.header[H_TICK])), recv=False)
                break
            meta = StepMeta.unpack(msg.header, msg.payload)
            out = stage.compute(meta, msg.data)
            if stage.is_last:
                # tail -> head: only the tokens (+ tick); the head still holds the metadata
                tmeta = StepMeta(kind=meta.kind, seq_ids=[], microbatch=meta.microbatch,
                                 step_id=meta.step_id)
                send = _msg_from(tmeta, out, int(msg.header[H_TICK]), tokens=True)
            elif out is None:
                send = _msg_from(meta, None, int(msg.header[H_TICK]), tokens=False)
            else:
                send = _msg_from(meta, out, int(msg.header[H_TICK]), tokens=False)
            msg = transport.exchange(send, recv=True)
        if kind == SHUTDOWN:
            return


# ------------------------------------------------------------------------------ builders
def build_stage(cfg: ModelConfig, rank: int, world: int, device, max_batch: int,
                max_model_len: int, block_size: int = 16, kv_fraction: float = 0.85,
                policy: str = "balanced", seed: int = 0, use_graphs=None,
                num_blocks: Optional[int] = None, dtype=torch.bfloat16):
    plans = plan_stages(cfg, world, policy)
    plan = plans[rank]
    table_width = -(-max_model_len // block_size)
    if num_blocks is None:
        cap = _stage_capacity_blocks(cfg, plan, block_size, device, kv_fraction,
                                     cap_tokens=max(world * max_batch * max_model_len, 1 << 16))
        t = torch.tensor([cap], dtype=torch.int64,
                         device=device if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MIN)     # block ids are global: same pool size
        num_blocks = int(t.item())
    stage = StageWorker(cfg, plan, device, num_blocks, block_size, max_batch, table_width,
                        seed=seed, use_graphs=use_graphs, dtype=dtype)
    return stage, plans, num_blocks, table_width


class DistributedPipelineEngine:
    """User-facing engine on rank 0 of an N-rank pipeline (ranks > 0 call ``serve()``)."""

    def __init__(self, model: str, device, max_batch: int = 256, max_model_len: int = 2048,
                 block_size: int = 16, policy: str = "balanced", seed: int = 0,
                 use_graphs=None, max_prefill_tokens: int = 16384, num_blocks=None,
                 dtype=torch.bfloat16):
        self.rank, self.world = init_distributed(device=torch.device(device)
                                                 if torch.device(device).type == "cuda" else None)
        self.cfg = get_config(model)
        self.device = torch.device(device)
        self.stage, self.plans, nb, tw = build_stage(
            self.cfg, self.rank, self.world, self.device, max_batch, max_model_len, block_size,
            policy=policy, seed=seed, use_graphs=use_graphs, num_blocks=num_blocks, dtype=dtype)
        self.transport = TorchDistTransport(self.device, self.cfg.hidden_size, dtype=dtype)
        self.head = None
        if self.rank == 0:
            bm = BlockManager(nb, block_size)
            sched = Scheduler(bm, max_seqs_per_mb=max_batch, max_prefill_tokens=max_prefill_tokens,
                              num_microbatches=self.world, eos_token_id=self.cfg.eos_token_id,
                              max_model_len=max_model_len, table_width=tw)
            self.head = PipelineHead(self.stage, self.transport, sched,
                                     load_tokenizer(self.cfg))
        self._ids = 0

    def warmup(self):
        self.stage.runner.capture()

    def add_request(self, prompt, params: Optional[SamplingParams] = None, request_id=None):
        assert self.head is not None, "requests enter at rank 0"
        rid = request_id or f"req-{self._ids}"
        self._ids += 1
        ids = self.head.tok.encode(prompt) if isinstance(prompt, str) else list(prompt)
        self.head.sched.add_request(rid, ids, params)
        return rid

    def generate(self, prompts, params=None) -> List[RequestOutput]:
        rids = [self.add_request(p, params) for p in prompts]
        outs = {o.request_id: o for o in self.head.run_session()}
        return [outs[r] for r in rids]

    def serve(self):
        """Non-head ranks: block serving sessions until the head shuts the ring down."""
        run_stage_loop(self.stage, self.transport)

    def shutdown(self):
        if self.head is not None:
            self.head.shutdown()


# ------------------------------------------------------------------------------ loopback
class LocalPipeline:
    """All N stages in one process (loopback transport): same partitioning, metadata
    serialisation and microbatch schedule as the distributed ring, executed sequentially."""

    def __init__(self, model, num_stages: int, device="cpu", max_batch: int = 64,
                 max_model_len: int = 512, block_size: int = 16, num_blocks: int = 256,
                 policy: str = "even", seed: int = 0, use_graphs=None, params=None,
                 dtype=torch.bfloat16, plans: Optional[List[StagePlan]] = None):
        self.cfg = get_config(model) if isinstance(model, str) else model
        self.N = num_stages
        self.plans = plans or plan_stages(self.cfg, num_stages, policy)
        tw = -(-max_model_len // block_size)
        self.stages = []
        for p in self.plans:
            sp = None
            if params is not None:
                sp = {k: v for k, v in params.items() if _param_in_stage(k, p, self.cfg)}
            self.stages.append(StageWorker(self.cfg, p, device, num_blocks, block_size,
                                           max_batch, tw, seed, use_graphs, params=sp,
                                           dtype=dtype))
        self.sched = Scheduler(BlockManager(num_blocks, block_size), max_seqs_per_mb=max_batch,
                               num_microbatches=num_stages, eos_token_id=self.cfg.eos_token_id,
                               max_model_len=max_model_len, table_width=tw)
        self.tok = load_tokenizer(self.cfg)
        self._ids = 0

    def generate(self, prompts, params=None) -> List[RequestOutput]:
        rids = []
        for p in prompts:
            rid = f"req-{self._ids}"
            self._ids += 1
            ids = self.tok.encode(p) if isinstance(p, str) else list(p)
            self.sched.add_request(rid, ids, params)
            rids.append(rid)
        k = 0
        inflight: Dict[int, tuple] = {}
        while self.sched.has_work() or inflight:
            j = k - self.N
            if j in inflight:
                m, toks = inflight.pop(j)
                self.sched.update(m, toks)
            meta = self.sched.schedule(k % self.N) if self.sched.has_work() else None
            if meta is not None:
                data = None
                for s in self.stages:
                    # round-trip the wire format exactly as the ring does
                    h, pl = meta.pack()
                    m2 = StepMeta.unpack(h, pl)
                    if not s.model.is_first:
                        m2.input_ids = None
                    data = s.compute(m2, data)
                inflight[k] = (meta, data.cpu().numpy())
            k += 1
        outs = {s.request_id: seq_to_output(s, self.tok) for s in self.sched.pop_finished()}
        return [outs[r] for r in rids]


def _param_in_stage(name: str, p: StagePlan, cfg: ModelConfig) -> bool:
    if name.startswith("layers."):
        i = int(name.split(".")[1])
        return p.start_layer <= i < p.end_layer
    if name in ("embed", "pos_embed"):
        return p.first or (p.last and cfg.tie_embeddings and name == "embed")
    return p.last


# ------------------------------------------------------------------------------ bench
def bench_pipeline(args, world: int, rank: int, make_prompts):
    """bench.py entry for N > 1: layer-sharded Llama-3-8B across the ranks of torchrun."""
    local = int(os.environ.get("LOCAL_RANK", rank))
    if os.environ.get("DLI_SAME_DEVICE", "0") == "1":
        local = 0          # rehearsal on a 1-GPU box: every rank computes on cuda:0 (gloo comm)
    if torch.cuda.is_available():
        torch.cuda.set_device(local)
        device = torch.device("cuda", local)
    else:
        device = torch.device("cpu")
    eng = DistributedPipelineEngine(args.model, device, max_batch=args.batch,
                                    max_model_len=args.max_model_len,
                                    max_prefill_tokens=max(args.batch * args.prompt_len, 8192))
    world = eng.world
    eng.warmup()
    sp = SamplingParams(max_length=args.max_length, temperature=0.8, top_k=50, top_p=0.95,
                        ignore_eos=True)
    per_wave = args.batch * world                  # N microbatches of --batch requests

    def wave(seed):
        if rank == 0:
            outs = eng.generate(make_prompts(per_wave, args.prompt_len, eng.cfg.vocab_size, seed),
                                sp)
            return sum(len(o.output_ids) for o in outs), [o.latency_s for o in outs]
        run_one_session(eng)
        return 0, []

    for w in range(args.warmup):
        wave(10_000 + w)
    dist.barrier()
    if device.type == "cuda":
        torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    toks, lats = 0, []
    for s in range(args.steps):
        n, l = wave(s)
        toks += n
        lats += l
    if device.type == "cuda":
        torch.cuda.synchronize(device)
    dist.barrier()
    dt = torch.tensor([time.perf_counter() - t0], dtype=torch.float64,
                      device=device if dist.get_backend() == "nccl" else "cpu")
    dist.all_reduce(dt, op=dist.ReduceOp.MAX)
    eng.shutdown() if rank == 0 else eng.serve()
    dist.barrier()
    dist.destroy_process_group()
    if rank != 0:
        return None
    return {"tokens": toks, "seconds": float(dt.item()), "latencies": lats,
            "global_batch": per_wave, "parallelism": f"pp{world}",
            "engine": eng.head.stats.snapshot()}


def run_one_session(eng: DistributedPipelineEngine):
    """Serve exactly one head session on a non-head rank (bench lockstep)."""
    tp, stage = eng.transport, eng.stage
    msg = tp.exchange(None, recv=True)
    while True:
        kind = int(msg.header[0])
        if kind in (STOP, SHUTDOWN):
            tp.exchange(_control(kind, int(msg.header[H_TICK])), recv=False)
            return
        meta = StepMeta.unpack(msg.header, msg.payload)
        out = stage.compute(meta, msg.data)
        if stage.is_last:
            tmeta = StepMeta(kind=meta.kind, seq_ids=[], microbatch=meta.microbatch,
                             step_id=meta.step_id)
            send = _msg_from(tmeta, out, int(msg.header[H_TICK]), tokens=True)
        else:
            send = _msg_from(meta, out, int(msg.header[H_TICK]), tokens=False)
        msg = tp.exchange(send, recv=True)
