"""Layer-sharded pipeline-parallel serving: one process per MI355X, stages over RCCL.

This is what the reference's "sharded inference" was meant to be (offline
layer split ``shard_model.py:55-109``, ``metadata.json``, ``/load_shard`` at
``worker/app.py:139-206``, dispatch to shard holders at ``master/dashboard/views.py:318-355``;
execution never actually coordinated the shards) — made real:

* stage r holds layers [start_r, end_r) (shard/planner.py, or the ``shard_<r>/`` files the
  ``shard-model`` CLI wrote, streamed into HBM by the C++ loader), its own paged KV pool
  and its own hipGraph-captured decode step;
* rank 0 (the head) owns the scheduler, the C++ block allocator and the tokenizer; each
  tick's packed step metadata is published once on the shared-memory control ring
  (``transport.py``), so the other stages hold no scheduling state at all;
* M = N + 1 microbatches circulate: while microbatch m is in stage r, stage r-1 runs the
  next one, so all N GPUs are busy in steady state; the tail samples on device and returns
  int32 tokens to the head (C3), which schedules that microbatch's next step a tick after
  they arrived (the extra microbatch keeps the head's host off the critical path);
* every receive lands in a buffer allocated once per engine (decode hidden states straight
  into the stage runner's static graph input); the tokens the head reads back travel
  through a ring of M pinned host slots: no tensor is allocated by the transport per tick;
* requests join a running session at tick boundaries (``run_session(admit=...)``), and
  finished requests are handed back the tick they finish;
* control plane (shared memory, host) / data plane (RCCL, stream-ordered): non-head ranks
  never synchronise their host with their GPU;
* sessions: the head drives ticks while it has work, then publishes STOP; other ranks
  block waiting for the next session; SHUTDOWN ends them.

``LocalPipeline`` runs the same partitioned stages and tick schedule in ONE process (all
stages on one device): the loopback transport used to test pipeline correctness on a single
GPU or CPU.
"""
from __future__ import annotations

import json
import os
import time
from pathlib import Path
from typing import Callable, Dict, List, Optional, Tuple

import numpy as np
import torch
import torch.distributed as dist

from ..engine.batch import DECODE, EMPTY, HEADER_LEN, PREFILL, STOP, StepMeta
from ..engine.kv_cache import KVCache, auto_num_blocks
from ..engine.llm_engine import EngineStats, seq_to_output
from ..engine.runner import StageRunner
from ..engine.scheduler import Scheduler
from ..engine.sequence import RequestOutput, SamplingParams
from .. import ops
from ..models import weights as W
from ..models.configs import ModelConfig, get_config
from ..models.model import TransformerLM
from ..runtime import BlockManager
from ..shard.planner import StagePlan, plan_stages
from ..tokenizer import load_tokenizer
from ..utils import faults
from .transport import H_TICK, PipeChannel, ctrl_slot_bytes, init_distributed

SHUTDOWN = 4


def _ctrl(kind: int, tick: int, meta: Optional[StepMeta] = None):
    if meta is None:
        h = np.zeros(HEADER_LEN, dtype=np.int64)
        h[0] = kind
        p = np.zeros(0, dtype=np.int32)
    else:
        h, p = meta.pack()
    h[H_TICK] = tick
    return h, p


def num_microbatches(world: int, vocab_parallel: bool = False) -> int:
    """Microbatches in flight. M = N + 1: the head re-schedules a microbatch one full tick
    after the tail returned its tokens, so no stage waits on the head's host (M = N would put
    the token sync + scheduling on the critical path of every tick). With the vocab-parallel
    head the tokens exist on rank 0 two ticks later (candidates, then sampling): M = N + 3."""
    if world <= 1:
        return 1
    return int(os.environ.get("DLI_PP_MICROBATCHES",
                              str(world + (3 if vocab_parallel else 1))))


def use_vocab_parallel(cfg: ModelConfig, world: int) -> bool:
    """Vocab-parallel LM head: every stage computes 1/N of the 1 GB Llama-3 head, which
    otherwise sits on the tail and (32 layers over 8 stages) leaves the 5-layer stages 17 %
    over the mean. DLI_PP_VOCAB_PARALLEL=0/1 forces it; default on for N >= 4."""
    env = os.environ.get("DLI_PP_VOCAB_PARALLEL", "auto")
    ok = world > 1 and not cfg.tie_embeddings and cfg.arch == "llama"
    if env in ("0", "1"):
        return ok and env == "1"
    return ok and world >= 4


CAND = 64          # per-rank candidates of the vocab-parallel LM head (max top_k served)


def vocab_slices(vocab: int, n: int) -> List[Tuple[int, int]]:
    b = [round(i * vocab / n) for i in range(n + 1)]
    return [(b[i], b[i + 1]) for i in range(n)]


class StageWorker:
    """Model slice + KV pool + hipGraph runner of one pipeline stage; with a vocab-parallel
    head also this rank's slice of the LM head (candidates) and, on rank 0, the sampler."""

    def __init__(self, cfg: ModelConfig, plan: StagePlan, device, num_blocks: int,
                 block_size: int, max_batch: int, table_width: int, seed: int = 0,
                 use_graphs: Optional[bool] = None, params=None, dtype=torch.bfloat16,
                 vocab_slice: Optional[Tuple[int, int]] = None, max_tokens: int = 0):
        self.cfg, self.plan = cfg, plan
        self.device = torch.device(device)
        self.max_batch = max_batch
        self.max_tokens = max(max_tokens, max_batch)
        if params is None:
            self.model = TransformerLM.random(cfg, plan.start_layer, plan.end_layer, self.device,
                                              dtype=dtype, seed=seed)
        else:
            self.model = TransformerLM(cfg, {k: v.to(self.device) for k, v in params.items()},
                                       plan.start_layer, plan.end_layer, self.device)
        self.vocab_parallel = vocab_slice is not None
        if self.vocab_parallel:
            lo, hi = vocab_slice
            if "head_slice" not in self.model.params:
                full = self.model.params.get("lm_head")
                if full is None:        # same per-name deterministic init as the tail's head
                    shape = W.stage_param_shapes(cfg, 0, cfg.num_layers, False, True)["lm_head"]
                    full = W.random_init({"lm_head": shape}, self.device, dtype, seed)["lm_head"]
                self.model.params["head_slice"] = full[lo:hi].contiguous()
                del full
            self.model.vocab_parallel = True
            self.model.vocab_offset = lo
        self.kv = KVCache(cfg, plan.end_layer - plan.start_layer, num_blocks, block_size,
                          self.device, dtype)
        self.runner = StageRunner(self.model, self.kv, max_batch, table_width, use_graphs)
        self.tick_counts: Dict[int, int] = {}     # non-head ranks: steps run, by kind
        self._samp = None                         # pinned staging ring of _sampling

    @property
    def is_last(self) -> bool:
        return self.model.is_last

    def compute(self, meta: StepMeta, data: Optional[torch.Tensor]) -> Optional[torch.Tensor]:
        """Layers of this stage. Last stage: int32 tokens, or with a vocab-parallel head the
        final normed hidden [S, D] of each sequence."""
        if meta.kind not in (PREFILL, DECODE) or meta.num_seqs == 0:
            return None
        return self.runner.run(meta, hidden=data)

    def _sampling(self, meta: StepMeta):
        """(temperature, top_k, top_p, seeds) of ``meta`` on the device. On a GPU they go
        through a ring of pinned staging buffers with async copies: a copy from pageable
        memory waits for everything queued on the stream, which put the head's host in
        lockstep with its GPU on every tick of the vocab-parallel head (rank 0's host time
        per decode tick was ~the whole tick, profiles/r6/README.md)."""
        d = self.device
        if d.type != "cuda":
            return (torch.from_numpy(np.ascontiguousarray(meta.temperature, np.float32)),
                    torch.from_numpy(np.ascontiguousarray(meta.top_k, np.int32)),
                    torch.from_numpy(np.ascontiguousarray(meta.top_p, np.float32)),
                    torch.from_numpy(np.ascontiguousarray(meta.seeds, np.int64)))
        S, B = meta.num_seqs, self.max_batch
        if self._samp is None:
            # layout (int32 words): seeds (2B, first: an int64 view needs an even offset) |
            # temperature (B) | top_k (B) | top_p (B)
            ring = [torch.zeros(5 * B, dtype=torch.int32).pin_memory() for _ in range(8)]
            self._samp = {"host": ring, "np": [t.numpy() for t in ring],
                          "ev": [torch.cuda.Event() for _ in ring], "used": [False] * 8,
                          "j": 0, "dev": torch.zeros(5 * B, dtype=torch.int32, device=d)}
        R = self._samp
        j = R["j"] = (R["j"] + 1) % len(R["host"])
        if R["used"][j]:
            R["ev"][j].synchronize()          # its copy 8 calls back: long done
        h = R["np"][j]
        h[:2 * S] = np.ascontiguousarray(meta.seeds, np.int64).view(np.int32)
        h[2 * B:2 * B + S] = np.ascontiguousarray(meta.temperature, np.float32).view(np.int32)
        h[3 * B:3 * B + S] = np.ascontiguousarray(meta.top_k, np.int32)
        h[4 * B:4 * B + S] = np.ascontiguousarray(meta.top_p, np.float32).view(np.int32)
        dev = R["dev"]
        dev.copy_(R["host"][j], non_blocking=True)
        R["ev"][j].record()
        R["used"][j] = True
        return (dev[2 * B:2 * B + S].view(torch.float32), dev[3 * B:3 * B + S],
                dev[4 * B:4 * B + S].view(torch.float32), dev[:2 * S].view(torch.int64))

    def candidates(self, hf: torch.Tensor) -> torch.Tensor:
        """This rank's top-CAND of its vocab slice, packed int32 [S, 2*CAND] (values | ids)."""
        v, i = self.model.head_candidates(hf, CAND)
        return torch.cat([v.contiguous().view(torch.int32), i], dim=1)

    def sample_candidates(self, meta: StepMeta, packed: List[torch.Tensor]) -> torch.Tensor:
        """Rank 0: merge every rank's candidates (rank order = ascending token ids) and
        sample with the request's warpers and Philox seed -> int32 tokens [S]."""
        vals = torch.cat([c[:, :CAND].contiguous().view(torch.float32) for c in packed], 1)
        ids = torch.cat([c[:, CAND:] for c in packed], 1).contiguous()
        return ops.sample(vals, *self._sampling(meta), ids=ids)

    def tokens_full(self, meta: StepMeta, hf: torch.Tensor) -> torch.Tensor:
        """Tail fallback (a row needs more than CAND candidates): full LM head + sampler."""
        return ops.sample(self.model.head_logits(hf), *self._sampling(meta))


def vp_ok(meta: Optional[StepMeta]) -> bool:
    """The vocab-parallel head serves a step when every row's top-k fits in CAND
    candidates per rank (greedy included); top_k <= 0 (full-vocab sampling) falls back."""
    if meta is None or meta.top_k is None or meta.num_seqs == 0:
        return False
    core = getattr(meta, "core", None)      # native decode step: rows' params are fixed and
    if core is not None:                    # rows only ever leave the core (compaction)
        st, _, S = core
        if st.vp is not None and st.vp[0] == S:
            return st.vp[1]
    tk = np.asarray(meta.top_k)
    greedy = np.asarray(meta.temperature) <= 0
    ok = bool(np.all(greedy | ((tk >= 1) & (tk <= CAND))))
    if core is not None:
        st.vp = (S, ok)
    return ok


H_VP = 13          # ctrl header word: 1 = vocab-parallel head for this step


def _stage_capacity_blocks(cfg, plan, block_size, device, kv_fraction, cap_tokens,
                           vocab_slice: Optional[Tuple[int, int]] = None,
                           loaded: bool = False):
    """KV blocks of this stage's pool, sized before its weights are loaded: the stage's own
    parameter bytes (plus its vocab-parallel head slice) are still to come, and with every
    rank on one device (``DLI_SAME_DEVICE=1``) so are every other rank's — summed over the
    ranks, or 8 ranks each sizing against the empty device over-commit it (Llama-3-70B pp8 on
    one GPU ran out of memory: profiles/r6/README.md)."""
    pending = 0
    if not loaded:                      # the shard-file path loads before sizing the pool
        shapes = W.stage_param_shapes(cfg, plan.start_layer, plan.end_layer, plan.first,
                                      plan.last)
        pending = sum(int(np.prod(s)) for s in shapes.values()) * 2
        if vocab_slice is not None:
            pending += (vocab_slice[1] - vocab_slice[0]) * cfg.hidden_size * 2
    if os.environ.get("DLI_SAME_DEVICE", "0") == "1" and dist.is_initialized():
        t = torch.tensor([pending], dtype=torch.int64)
        dist.all_reduce(t, group=_cpu_group())
        pending = int(t.item())
    return auto_num_blocks(cfg, plan.end_layer - plan.start_layer, block_size, device,
                           kv_fraction, cap_tokens=cap_tokens, pending_bytes=pending)


_CPU_GROUP = None


def _cpu_group():
    """A gloo group over every rank (host-side sums when the default group is RCCL)."""
    global _CPU_GROUP
    if _CPU_GROUP is None:
        from datetime import timedelta
        _CPU_GROUP = (dist.group.WORLD if dist.get_backend() == "gloo"
                      else dist.new_group(backend="gloo", timeout=timedelta(minutes=30)))
    return _CPU_GROUP


class _TokenRing:
    """The head's view of each microbatch's sampled ids: M device slots (the tail's tokens
    land here, or rank 0's own sampler output is parked here) mirrored into M pinned host
    slots by an async D2H copy + event, enqueued right behind the producing step. Slot
    = start tick % M: a microbatch's slot is refilled only after the host consumed it."""

    def __init__(self, ch: PipeChannel, M: int, max_batch: int):
        self.M = M
        self.dev = ch.recv_buffer((M, max_batch), torch.int32)
        self.cuda = self.dev.is_cuda
        if self.cuda:
            self.host = torch.empty((M, max_batch), dtype=torch.int32, pin_memory=True)
            self.ev = [torch.cuda.Event() for _ in range(M)]
        self.n = [0] * M
        self.rows = list(self.dev.unbind(0))          # per-slot views, made once
        self.host_rows = list(self.host.unbind(0)) if self.cuda else None

    def slot(self, start_tick: int, n: int) -> torch.Tensor:
        return self.rows[start_tick % self.M][:n]

    def landed(self, start_tick: int, n: int, src: Optional[torch.Tensor] = None) -> None:
        """Tokens of microbatch ``start_tick`` are in (or, with ``src``, copied into) their
        device slot: start the host copy."""
        j = start_tick % self.M
        row = self.rows[j]
        if src is not None and src.data_ptr() != row.data_ptr():
            if src.device != row.device:
                src = src.to(row.device)
            row[:n].copy_(src if src.shape[0] == n else src[:n], non_blocking=True)
        self.n[j] = n
        if self.cuda:
            self.host_rows[j][:n].copy_(row[:n], non_blocking=True)
            self.ev[j].record()

    def get(self, start_tick: int) -> np.ndarray:
        j = start_tick % self.M
        if self.cuda:
            self.ev[j].synchronize()
            return self.host_rows[j][:self.n[j]].numpy()
        return self.rows[j][:self.n[j]].numpy()


class PipelineHead:
    """Rank-0 driver: scheduler + tick loop over M microbatches (stage 0 is also this rank).

    Tick k (all ranks exchange once, anti-diagonal: rank r runs the layers of the microbatch
    the head started at tick k - r):
      consume tokens of the microbatch started at k - M, admit newly arrived requests,
      schedule that microbatch's next step, publish the step's metadata (control plane),
      post exchange(k), then
        vocab-parallel head: candidates of microbatch k - N from its final hidden (received
          from the tail); merge every rank's candidates of microbatch k - 1 - N and sample;
        tail head (fallback): tokens of microbatch k - N arrive from the tail;
      and run stage 0's layers for tick k. M = N + 3 with the vocab-parallel head (tokens
      exist on rank 0 one tick after the candidates), N + 1 otherwise."""

    def __init__(self, stage: StageWorker, channel, scheduler: Scheduler, tokenizer,
                 microbatches: Optional[int] = None):
        self.stage, self.ch, self.sched, self.tok = stage, channel, scheduler, tokenizer
        self.N = channel.world
        self.vp = stage.vocab_parallel
        self.M = microbatches or num_microbatches(self.N, self.vp)
        assert self.N == 1 or self.M >= self.N + (3 if self.vp else 1), "too few microbatches"
        self.stats = EngineStats()
        self.host_s = 0.0          # head host time in ticks, excluding transport waits
        self.ticks = 0
        self.tick_log = [] if os.environ.get("DLI_PP_TICK_LOG", "0") == "1" else None
        # host seconds / ticks by step kind (EMPTY / PREFILL / DECODE)
        self.host_by_kind = {EMPTY: [0.0, 0], PREFILL: [0.0, 0], DECODE: [0.0, 0]}
        self.phase_s = {k: 0.0 for k in ("update", "finish", "schedule", "ctrl", "head_ops",
                                         "compute")}
        B, D = stage.max_batch, stage.cfg.hidden_size
        self.tokens = _TokenRing(channel, self.M, B)
        if self.vp and self.N > 1:
            self.hf_rx = channel.recv_buffer((B, D))
            self.cand_rx = channel.recv_buffer((self.N - 1, B, 2 * CAND), torch.int32)
        # row-count -> views of the receive buffers (a decode microbatch keeps its row count
        # for many ticks; slicing 2N tensors per tick is ~4 us each on the head's host)
        self._hf_views: Dict[int, torch.Tensor] = {}
        self._cand_views: Dict[int, List[torch.Tensor]] = {}

    def _hf_view(self, S: int) -> torch.Tensor:
        v = self._hf_views.get(S)
        if v is None:
            v = self._hf_views[S] = self.hf_rx[:S]
        return v

    def _cand_view(self, S: int) -> List[torch.Tensor]:
        v = self._cand_views.get(S)
        if v is None:
            v = self._cand_views[S] = [self.cand_rx[q, :S] for q in range(self.N - 1)]
        return v

    def _account(self, meta: StepMeta):
        self.stats.steps += 1
        if meta.kind == PREFILL:
            self.stats.prefill_steps += 1
            self.stats.prompt_tokens += meta.num_tokens
        else:
            self.stats.decode_steps += 1

    def _finished(self) -> List[RequestOutput]:
        outs = []
        for seq in self.sched.pop_finished():
            o = seq_to_output(seq, self.tok)
            self.stats.finished += 1
            self.stats.latencies.append(o.latency_s)
            outs.append(o)
        return outs

    def run_session(self, admit: Optional[Callable[[], int]] = None,
                    on_finished: Optional[Callable[[List[RequestOutput]], None]] = None
                    ) -> List[RequestOutput]:
        """Drive ticks until nothing is queued, running or in flight. ``admit`` is called
        at every tick boundary to add newly arrived requests to the scheduler (continuous
        admission); ``on_finished`` receives the requests that finished at that tick (else
        everything is returned at the end)."""
        N, M, k, ch, st = self.N, self.M, 0, self.ch, self.stage
        started: Dict[int, Tuple[StepMeta, bool]] = {}   # start tick -> (meta, vocab-parallel)
        prev_out = None                # stage-0 output of tick k-1 (hidden -> rank 1)
        my_cand = None                 # own candidates of microbatch k-1-N (vocab-parallel)
        collected: List[RequestOutput] = []
        toks = self.tokens
        ph = self.phase_s
        pc = time.perf_counter
        tt = time.thread_time       # this thread's CPU time: host cost without preemption
        # every plane: a dead peer seen by the watchdog (any plane) or the device mailboxes'
        # error word (ipc) fails the session at the next tick boundary
        check = getattr(ch, "check", None) if N > 1 else None
        while True:
            t0 = pc()
            c0 = tt()
            wait_s = wait_c = 0.0
            if check is not None:
                check()                      # device data plane healthy (one host load)
            s = k - M
            if s in started:
                m, _ = started.pop(s)
                arr = toks.get(s)
                tw = pc()
                wait_s += tw - t0
                self.sched.update(m, arr)
                self.stats.tokens_out += m.num_sampled
                ph["update"] += pc() - tw
            t1 = pc()
            if admit is not None:
                admit()
            done = self._finished()
            if done:
                if on_finished is not None:
                    on_finished(done)
                else:
                    collected += done
            t2 = pc()
            ph["finish"] += t2 - t1
            meta = self.sched.schedule(k % M) if self.sched.has_work() else None
            t3 = pc()
            ph["schedule"] += t3 - t2
            if meta is None and not started and not self.sched.has_work():
                break
            if N == 1:
                if meta is not None:
                    out = st.compute(meta, None)
                    started[k] = (meta, False)
                    toks.landed(k, meta.num_seqs, src=out)
                    self._account(meta)
                k += 1
                continue
            vp_k = self.vp and vp_ok(meta)
            h, p = _ctrl(EMPTY if meta is None else meta.kind, k, meta)
            h[H_VP] = int(vp_k)
            ch.broadcast_ctrl(h, p)
            t4 = pc()
            ph["ctrl"] += t4 - t3
            ret = started.get(k - N)             # its last stage ran at tick k - 1
            smp = started.get(k - 1 - N)         # its candidates were made at tick k - 1
            recvs = []
            if ret is not None:
                S = ret[0].num_seqs
                recvs.append((self._hf_view(S), N - 1, 2) if ret[1] else
                             (toks.slot(k - N, S), N - 1, 2))
            if smp is not None and smp[1]:
                cv = self._cand_view(smp[0].num_seqs)
                recvs += [(cv[q - 1], q, 3) for q in range(1, N)]
            tw, cw = pc(), tt()
            ch.exchange([(prev_out, 1, 1)] if prev_out is not None else [], recvs)
            ch.reap_ctrl()
            t5 = pc()
            wait_s += t5 - tw
            wait_c += tt() - cw
            cand_now = None
            if ret is not None:
                if ret[1]:
                    cand_now = st.candidates(ch.to_compute(self._hf_view(ret[0].num_seqs)))
                else:
                    toks.landed(k - N, ret[0].num_seqs)
            if smp is not None and smp[1]:
                S2 = smp[0].num_seqs
                cv = self._cand_view(S2)
                bufs = cv if ch.data_device == ch.device else [ch.to_compute(b) for b in cv]
                tok = st.sample_candidates(smp[0], [my_cand] + bufs)
                toks.landed(k - 1 - N, S2, src=tok)
            my_cand = cand_now
            prev_out = None
            t6 = pc()
            ph["head_ops"] += t6 - t5
            if meta is not None:
                prev_out = st.compute(meta, None)
                started[k] = (meta, vp_k)
                self._account(meta)
            now = pc()
            ph["compute"] += now - t6
            hs = now - t0 - wait_s
            kk = self.host_by_kind[meta.kind if meta is not None else EMPTY]
            kk[0] += hs
            kk[1] += 1
            if self.tick_log is not None:
                self.tick_log.append((meta.kind if meta is not None else 0, hs,
                                      t2 - t1, t3 - t2, t4 - t3, t6 - t5, now - t6,
                                      tt() - c0 - wait_c))
            self.host_s += hs
            self.ticks += 1
            self.stats.busy_s += now - t0
            k += 1
        if N > 1:
            ch.broadcast_ctrl(*_ctrl(STOP, k))
            ch.flush()
        done = self._finished()
        if on_finished is not None and done:
            on_finished(done)
        return collected + done

    def shutdown(self):
        if self.N > 1:
            self.ch.broadcast_ctrl(*_ctrl(SHUTDOWN, -1))
            self.ch.flush()


class _StageBuffers:
    """Receive buffers of a non-head stage, allocated once: hidden rows from the previous
    stage (prefill-sized; decode steps land in the runner's static graph input instead) and,
    with the vocab-parallel head, the tail's final hidden state."""

    def __init__(self, stage: StageWorker, ch: PipeChannel):
        D = stage.cfg.hidden_size
        self.rx = ch.recv_buffer((stage.max_tokens, D))
        self.hf = (ch.recv_buffer((stage.max_batch, D))
                   if stage.vocab_parallel and not stage.is_last else None)
        self.direct = ch.nccl or stage.device.type == "cpu" or ch.ipc is not None

    def hidden_target(self, stage: StageWorker, meta: StepMeta) -> torch.Tensor:
        if self.direct:
            b = stage.runner.input_buffer(meta)
            if b is not None:
                return b
        T = meta.num_tokens
        if T > self.rx.shape[0]:
            raise ValueError(f"step of {T} tokens exceeds the stage receive buffer "
                             f"({self.rx.shape[0]}); raise max_prefill_tokens")
        return self.rx[:T]


def install_piped(stage: StageWorker, channel) -> bool:
    """IPC data plane on a non-head GPU stage: capture the stage's receive (from r - 1) and
    send (to r + 1; on a tail without the vocab-parallel head, its sampled tokens to rank 0)
    INTO its decode graphs, so a decode tick costs one metadata H2D + one graph launch. The
    mailbox semaphores inside a captured graph are wait / signal kernels
    (csrc/runtime/ipc.cpp), which replay correctly: the per-edge sequence numbers live on the
    device and the put / get kernels advance them on every replay."""
    r, N = channel.rank, channel.world
    run = stage.runner
    if (channel.ipc is None or r == 0 or not run.use_graphs or run.hidden_in is None
            or os.environ.get("DLI_PP_SCHEDULE", "piped") == "grouped"):
        return False
    tail = r == N - 1
    if tail and stage.vocab_parallel:
        post = None                  # its per-step output (hf / fallback tokens) goes eagerly
    elif tail:
        def post(b, out):
            channel.exchange([(out[:b], 0, 2)], [])
    else:
        def post(b, out):
            channel.exchange([(out[:b], r + 1, 1)], [])

    def pre(b):
        channel.exchange([], [(run.hidden_in[:b], r - 1, 1)])
    run.set_piped(pre, post)
    return True


def _serve_session_piped(stage: StageWorker, channel, bufs: _StageBuffers) -> int:
    """``serve_session`` on the mailbox data plane (FIFO per edge, one message buffered per
    edge): tick k = [side messages: this rank's candidates -> 0, the tail's deferred output;
    the tail's final hidden <- N-1] then [receive x <- r-1, layers, send -> r+1] — the second
    bracket is ONE graph replay on decode ticks (``install_piped``), the same three
    operations issued eagerly on prefill ticks. Every wait depends on an earlier tick of a
    peer, so the schedule cannot deadlock; the tag-blind CPU model of the mailboxes
    (``fifo.py``) runs it at N = 2..8 in tests/test_fifo_transport.py."""
    r, N, k = channel.rank, channel.world, 0
    tail = r == N - 1
    run = stage.runner
    counts = stage.tick_counts
    metas: Dict[int, Tuple[StepMeta, bool]] = {}
    prev_out = None                 # tail + vocab-parallel head: my output of tick k-1
    prev_vp = False
    my_cand = None
    chk = getattr(channel, "check", None)
    while True:
        if faults.active():
            faults.check("pipeline.stage", tick=k)
        if chk is not None:
            chk()                            # device data plane healthy (one host load)
        meta = None
        if k >= r:
            h, p = channel.recv_ctrl()
            kind = int(h[0])
            if kind in (STOP, SHUTDOWN):
                channel.flush()
                return kind
            if kind in (PREFILL, DECODE):
                meta = StepMeta.unpack(h, p)
                metas[k - r] = (meta, bool(h[H_VP]))
        ret = metas.get(k - N)
        smp = metas.get(k - 1 - N)
        sends, recvs = [], []
        if tail and prev_out is not None:
            sends += ([(prev_out, q, 2) for q in range(N - 1)] if prev_vp
                      else [(prev_out, 0, 2)])
        if smp is not None and smp[1] and my_cand is not None:
            sends.append((my_cand, 0, 3))
        hf = None
        if ret is not None and ret[1] and not tail:
            hf = bufs.hf[:ret[0].num_seqs]
            recvs.append((hf, N - 1, 2))
        if sends or recvs:
            channel.exchange(sends, recvs)
        cand_now = None
        if ret is not None and ret[1]:
            cand_now = stage.candidates(prev_out if tail else hf)
        my_cand = cand_now
        prev_out, prev_vp = None, False
        if meta is not None:
            counts[meta.kind] = counts.get(meta.kind, 0) + 1
            vp_m = metas[k - r][1]
            if run.piped is not None and run.input_buffer(meta) is not None:
                out = stage.compute(meta, None)            # receive + layers + send: 1 graph
                if tail and stage.vocab_parallel:
                    if not vp_m:
                        out = stage.tokens_full(meta, out)
                    prev_out, prev_vp = out, vp_m
            else:
                x = bufs.rx[:meta.num_tokens]
                if x.shape[0] < meta.num_tokens:
                    raise ValueError(f"step of {meta.num_tokens} tokens exceeds the stage "
                                     f"receive buffer ({bufs.rx.shape[0]})")
                channel.exchange([], [(x, r - 1, 1)])
                out = stage.compute(meta, x)
                if tail and not vp_m and stage.vocab_parallel:
                    out = stage.tokens_full(meta, out)
                if not tail:
                    channel.exchange([(out, r + 1, 1)], [])
                elif not stage.vocab_parallel:
                    channel.exchange([(out, 0, 2)], [])
                else:
                    prev_out, prev_vp = out, vp_m
        for old in [t for t in metas if t < k - 1 - N]:
            del metas[old]
        k += 1


def serve_session(stage: StageWorker, channel, bufs: Optional[_StageBuffers] = None) -> int:
    """Non-head rank r: every tick of one head session; returns STOP or SHUTDOWN.
    Tick k: layers of the microbatch started at k - r (control message k - r, received in
    order), with the vocab-parallel head also the candidates of microbatch k - N; the tail
    returns either its final hidden (to every rank) or its sampled tokens (to rank 0). The
    host never waits on this GPU: receives, replays and sends are all stream-ordered."""
    bufs = bufs or _StageBuffers(stage, channel)
    # the mailbox plane runs the piped schedule; DLI_PP_SCHEDULE=grouped runs THIS (the
    # torch / RCCL) schedule over it instead, so the tag-blind FIFO model of the mailboxes
    # (fifo.py) checks the grouped schedule's message order too (tests/test_fifo_transport.py)
    if channel.ipc is not None and os.environ.get("DLI_PP_SCHEDULE", "piped") != "grouped":
        return _serve_session_piped(stage, channel, bufs)
    r, N, k = channel.rank, channel.world, 0
    tail = r == N - 1
    metas: Dict[int, Tuple[StepMeta, bool]] = {}
    prev_out = None                 # my layer output of tick k-1 (hidden / tokens / final hidden)
    prev_vp = False
    my_cand = None                  # my candidates of microbatch k-1-N
    chk = getattr(channel, "check", None)
    while True:
        if faults.active():
            faults.check("pipeline.stage", tick=k)
        if chk is not None:
            chk()                            # a dead peer fails the session here
        meta = None
        if k >= r:
            h, p = channel.recv_ctrl()
            kind = int(h[0])
            if kind in (STOP, SHUTDOWN):
                channel.flush()
                return kind
            if kind in (PREFILL, DECODE):
                meta = StepMeta.unpack(h, p)
                metas[k - r] = (meta, bool(h[H_VP]))
        ret = metas.get(k - N)
        smp = metas.get(k - 1 - N)
        sends, recvs = [], []
        if not tail and prev_out is not None:
            sends.append((prev_out, r + 1, 1))
        if tail and prev_out is not None:
            if prev_vp:
                sends += [(prev_out, q, 2) for q in range(N - 1)]
            else:
                sends.append((prev_out, 0, 2))
        if smp is not None and smp[1] and my_cand is not None:
            sends.append((my_cand, 0, 3))
        x = None
        if meta is not None:
            x = bufs.hidden_target(stage, meta)
            recvs.append((x, r - 1, 1))
        hf = None
        if ret is not None and ret[1] and not tail:
            hf = bufs.hf[:ret[0].num_seqs]
            recvs.append((hf, N - 1, 2))
        channel.exchange(sends, recvs)
        # candidates first: on the tail they read the final hidden of tick k-1 (prev_out),
        # which this tick's replay overwrites
        cand_now = None
        if ret is not None and ret[1]:
            cand_now = stage.candidates(prev_out if tail else channel.to_compute(hf))
        my_cand = cand_now
        prev_out, prev_vp = None, False
        if meta is not None:
            out = stage.compute(meta, channel.to_compute(x))
            vp_m = metas[k - r][1]
            if tail and not vp_m and stage.vocab_parallel:
                out = stage.tokens_full(meta, out)        # a row needs the whole vocabulary
            prev_out, prev_vp = out, vp_m
        for old in [t for t in metas if t < k - 1 - N]:
            del metas[old]
        k += 1


def run_stage_loop(stage: StageWorker, channel) -> None:
    """Non-head ranks: serve sessions until SHUTDOWN."""
    bufs = _StageBuffers(stage, channel)
    while serve_session(stage, channel, bufs) != SHUTDOWN:
        pass


# ------------------------------------------------------------------------------ shard files
def read_shard_dir(shard_dir: str, rank: int, world: int) -> Tuple[ModelConfig, dict, Path]:
    """(config, metadata, path) of ``<shard_dir>/shard_<rank>`` as written by ``shard-model``
    (reference layout); the files' partition must have ``world``
    stages."""
    d = Path(shard_dir) / f"shard_{rank}"
    meta = json.loads((d / "metadata.json").read_text())
    if int(meta.get("num_shards", 1)) != world:
        raise ValueError(f"{shard_dir} holds {meta.get('num_shards')} shards; the pipeline "
                         f"has {world} ranks")
    if int(meta.get("shard_id", rank)) != rank:
        raise ValueError(f"{d}: metadata.json says shard {meta.get('shard_id')}")
    cfg = ModelConfig.from_dict(json.loads((d / "config.json").read_text()))
    return cfg, meta, d


def load_stage_params(shard_dir: str, rank: int, world: int, device,
                      vocab_slice: Optional[Tuple[int, int]] = None) -> Dict[str, torch.Tensor]:
    """This rank's tensors straight from its shard file into HBM (C++ loader: mmap ->
    pinned ring -> hipMemcpyAsync). With the vocab-parallel head the rank also reads its
    row slice of the LM head from the last shard's file (a contiguous byte range)."""
    from ..runtime import SafetensorsFile
    _cfg, _meta, d = read_shard_dir(shard_dir, rank, world)
    f = SafetensorsFile(str(d / "model.safetensors"))
    try:
        params = f.load(device=device)
    finally:
        f.close()
    if vocab_slice is not None:
        tail = Path(shard_dir) / f"shard_{world - 1}" / "model.safetensors"
        ft = SafetensorsFile(str(tail))
        try:
            params["head_slice"] = ft.load_rows("lm_head", *vocab_slice, device=device)
        finally:
            ft.close()
    if torch.device(device).type == "cuda":
        torch.cuda.synchronize(device)
    return params


# ------------------------------------------------------------------------------ builders
def build_stage(cfg: ModelConfig, rank: int, world: int, device, max_batch: int,
                max_model_len: int, block_size: int = 16, kv_fraction: float = 0.85,
                policy: str = "balanced", seed: int = 0, use_graphs=None,
                num_blocks: Optional[int] = None, dtype=torch.bfloat16,
                vocab_parallel: bool = False, microbatches: Optional[int] = None,
                max_tokens: int = 0, shard_dir: Optional[str] = None,
                max_kv_tokens: int = 0):
    if shard_dir is not None:
        from ..shard.writer import stage_plan_from_metadata
        plans = [stage_plan_from_metadata(read_shard_dir(shard_dir, i, world)[1])
                 for i in range(world)]
    else:
        plans = plan_stages(cfg, world, policy, head_on_all=vocab_parallel)
    plan = plans[rank]
    table_width = -(-max_model_len // block_size)
    M = microbatches or num_microbatches(world, vocab_parallel)
    vs = vocab_slices(cfg.vocab_size, world)[rank] if vocab_parallel else None
    params = (load_stage_params(shard_dir, rank, world, device, vs)
              if shard_dir is not None else None)
    if num_blocks is None:
        # this stage's layers' KV from its free HBM (288 GB per MI355X); every stage holds
        # the same block ids (the head's allocator), so all take the smallest pool
        cap = _stage_capacity_blocks(cfg, plan, block_size, device, kv_fraction,
                                     cap_tokens=max_kv_tokens, vocab_slice=vs,
                                     loaded=params is not None)
        t = torch.tensor([cap], dtype=torch.int64,
                         device=device if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MIN)     # block ids are global: same pool size
        num_blocks = int(t.item())
    stage = StageWorker(cfg, plan, device, num_blocks, block_size, max_batch, table_width,
                        seed=seed, use_graphs=use_graphs, dtype=dtype, vocab_slice=vs,
                        max_tokens=max_tokens, params=params)
    return stage, plans, num_blocks, table_width


class DistributedPipelineEngine:
    """User-facing engine on rank 0 of an N-rank pipeline (ranks > 0 call ``serve()``).
    ``shard_dir``: serve the weights the ``shard-model`` CLI exported (one
    ``shard_<rank>/`` per rank) instead of a random init."""

    def __init__(self, model: str, device, max_batch: int = 256, max_model_len: int = 2048,
                 block_size: int = 16, policy: str = "balanced", seed: int = 0,
                 use_graphs=None, max_prefill_tokens: int = 16384, num_blocks=None,
                 dtype=torch.bfloat16, vocab_parallel: Optional[bool] = None,
                 shard_dir: Optional[str] = None, max_kv_tokens: int = 0):
        self.rank, self.world = init_distributed(device=torch.device(device)
                                                 if torch.device(device).type == "cuda" else None)
        if shard_dir is not None:
            self.cfg = read_shard_dir(shard_dir, self.rank, self.world)[0]
        else:
            self.cfg = get_config(model)
        self.device = torch.device(device)
        self.vocab_parallel = (use_vocab_parallel(self.cfg, self.world)
                               if vocab_parallel is None else vocab_parallel)
        self.microbatches = num_microbatches(self.world, self.vocab_parallel)
        max_model_len = min(max_model_len, self.cfg.max_position)
        # mixed steps (DLI_MIXED_STEPS, default on): a prefill step of a microbatch that is
        # decoding also carries that microbatch's decode rows (one token each), so its
        # running sequences do not sit out the admission; such a step holds up to
        # max_prefill_tokens + max_batch tokens (every rank sizes for it, whatever the head
        # decides)
        self.mixed_steps = os.environ.get("DLI_MIXED_STEPS", "1") == "1"
        max_tokens = max(max_prefill_tokens + max_batch, max_model_len)
        self.stage, self.plans, nb, tw = build_stage(
            self.cfg, self.rank, self.world, self.device, max_batch, max_model_len, block_size,
            policy=policy, seed=seed, use_graphs=use_graphs, num_blocks=num_blocks, dtype=dtype,
            vocab_parallel=self.vocab_parallel, microbatches=self.microbatches,
            max_tokens=max_tokens, shard_dir=shard_dir, max_kv_tokens=max_kv_tokens)
        esz = torch.empty(0, dtype=dtype).element_size()
        D = self.cfg.hidden_size
        # mailbox sizes of the IPC data plane: a whole step's hidden rows on r -> r + 1; the
        # tail's final hidden / tokens and the candidates on every other edge
        self.channel = PipeChannel(self.device, dtype=dtype,
                                   ctrl_bytes=ctrl_slot_bytes(max_batch, max_tokens, tw),
                                   msg_bytes=(max_tokens * D * esz,
                                              max(max_batch * D * esz, max_batch * 8 * CAND)))
        self.head = None
        if self.rank == 0:
            bm = BlockManager(nb, block_size)
            sched = Scheduler(bm, max_seqs_per_mb=max_batch, max_prefill_tokens=max_prefill_tokens,
                              num_microbatches=self.microbatches,
                              eos_token_id=self.cfg.eos_token_id,
                              max_model_len=max_model_len, table_width=tw,
                              native_decode=os.environ.get("DLI_NATIVE_SCHED", "1") == "1",
                              mixed_steps=self.mixed_steps)
            tok_path = None
            if shard_dir is not None and (Path(shard_dir) / "tokenizer").exists():
                tok_path = str(Path(shard_dir) / "tokenizer")
            self.head = PipelineHead(self.stage, self.channel, sched,
                                     load_tokenizer(self.cfg, tok_path), self.microbatches)
        self._ids = 0

    def warmup(self):
        install_piped(self.stage, self.channel)
        run = self.stage.runner
        if (run.use_graphs and os.environ.get("DLI_GEMM_AUTOTUNE", "1") == "1"
                and getattr(self.channel, "ctrl_group", None) is not None):
            # tune every bucket, then barrier, then capture: a stage's captured exchange
            # never waits on a peer that is still tuning (ranks sharing a GPU tune one at a
            # time, StageRunner.tune_lock)
            run.autotune(run.buckets)
            dist.barrier(group=self.channel.ctrl_group)
        run.capture()
        self.channel.start_watchdog()

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
        run_stage_loop(self.stage, self.channel)

    def shutdown(self):
        if self.head is not None:
            self.head.shutdown()


# ------------------------------------------------------------------------------ loopback
class LocalPipeline:
    """All N stages in one process (loopback transport): same partitioning, metadata
    serialisation and microbatch schedule as the distributed ring, executed sequentially.
    ``step()`` advances one tick, so a service can admit requests between ticks."""

    def __init__(self, model, num_stages: int, device="cpu", max_batch: int = 64,
                 max_model_len: int = 512, block_size: int = 16, num_blocks: int = 256,
                 policy: str = "even", seed: int = 0, use_graphs=None, params=None,
                 dtype=torch.bfloat16, plans: Optional[List[StagePlan]] = None,
                 stage_params: Optional[List[Dict[str, torch.Tensor]]] = None, tokenizer=None):
        self.cfg = get_config(model) if isinstance(model, str) else model
        self.N = num_stages
        self.plans = plans or plan_stages(self.cfg, num_stages, policy)
        tw = -(-max_model_len // block_size)
        self.stages = []
        for i, p in enumerate(self.plans):
            sp = None
            if stage_params is not None:
                sp = stage_params[i]
            elif params is not None:
                sp = {k: v for k, v in params.items() if _param_in_stage(k, p, self.cfg)}
            self.stages.append(StageWorker(self.cfg, p, device, num_blocks, block_size,
                                           max_batch, tw, seed, use_graphs, params=sp,
                                           dtype=dtype))
        self.sched = Scheduler(BlockManager(num_blocks, block_size), max_seqs_per_mb=max_batch,
                               num_microbatches=num_stages, eos_token_id=self.cfg.eos_token_id,
                               max_model_len=max_model_len, table_width=tw,
                               native_decode=os.environ.get("DLI_NATIVE_SCHED", "1") == "1")
        self.tok = tokenizer or load_tokenizer(self.cfg)
        self.stats = EngineStats()
        self._ids = 0
        self._k = 0
        self._inflight: Dict[int, tuple] = {}

    def add_request(self, prompt, params=None, request_id=None) -> str:
        rid = request_id or f"req-{self._ids}"
        self._ids += 1
        ids = self.tok.encode(prompt) if isinstance(prompt, str) else list(prompt)
        self.sched.add_request(rid, ids, params)
        return rid

    def has_work(self) -> bool:
        return self.sched.has_work() or bool(self._inflight)

    def step(self) -> List[RequestOutput]:
        """One tick: apply the tokens of the microbatch started N ticks ago, schedule the
        next step of this tick's microbatch and run it through every stage."""
        k, N = self._k, self.N
        t0 = time.perf_counter()
        j = k - N
        if j in self._inflight:
            m, toks = self._inflight.pop(j)
            self.sched.update(m, toks)
            self.stats.tokens_out += m.num_sampled
        meta = self.sched.schedule(k % N) if self.sched.has_work() else None
        if meta is not None:
            data = None
            for s in self.stages:
                # round-trip the wire format exactly as the ring does
                h, pl = meta.pack()
                m2 = StepMeta.unpack(h, pl)
                if not s.model.is_first:
                    m2.input_ids = None
                data = s.compute(m2, data)
            self._inflight[k] = (meta, data.cpu().numpy())
            self.stats.steps += 1
            if meta.kind == PREFILL:
                self.stats.prefill_steps += 1
            else:
                self.stats.decode_steps += 1
            self.stats.busy_s += time.perf_counter() - t0
        self._k += 1
        outs = []
        for s in self.sched.pop_finished():
            o = seq_to_output(s, self.tok)
            self.stats.finished += 1
            self.stats.latencies.append(o.latency_s)
            outs.append(o)
        return outs

    def generate(self, prompts, params=None) -> List[RequestOutput]:
        rids = [self.add_request(p, params) for p in prompts]
        outs: Dict[str, RequestOutput] = {}
        while self.has_work():
            for o in self.step():
                outs[o.request_id] = o
        for o in self.step():
            outs[o.request_id] = o
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
    # prefill admission in C steps per microbatch (bench --pp-prefill-chunks, default 2): the
    # wave starts with every stage filling the ring, and stage r idles r ticks of prefill
    # length — the GPipe bubble (N-1)/(C*M+N-1) of the prefill phase. At N = 8 (M = 11, a
    # 16k-token prefill tick ~21 ms on a 4-layer stage) one step per microbatch idles ~150 ms
    # per ~1.3 s wave; two steps of 8k tokens halve that. Decode ticks are unchanged.
    chunks = max(1, int(getattr(args, "pp_prefill_chunks", 2)))
    eng = DistributedPipelineEngine(args.model, device, max_batch=args.batch,
                                    max_model_len=args.max_model_len,
                                    max_prefill_tokens=max(args.batch * args.prompt_len // chunks,
                                                           4096),
                                    shard_dir=getattr(args, "shard_dir", None))
    world = eng.world
    t_w = time.perf_counter()
    eng.warmup()
    if rank == 0:
        import sys as _sys
        print(f"[bench] pp{world} engine warm-up (autotune + capture): "
              f"{time.perf_counter() - t_w:.1f} s", file=_sys.stderr, flush=True)
    sp = SamplingParams(max_length=args.max_length, temperature=0.8, top_k=50, top_p=0.95,
                        ignore_eos=True)
    per_wave = args.batch * eng.microbatches       # M microbatches of --batch requests
    bufs = None if rank == 0 else _StageBuffers(eng.stage, eng.channel)

    def wave(seed):
        if rank == 0:
            outs = eng.generate(make_prompts(per_wave, args.prompt_len, eng.cfg.vocab_size, seed),
                                sp)
            return sum(len(o.output_ids) for o in outs), [o.latency_s for o in outs]
        serve_session(eng.stage, eng.channel, bufs)
        return 0, []

    def progress(what, i, n, t):
        if rank == 0:
            import sys as _sys
            print(f"[bench] pp{world} {what} wave {i + 1}/{n}: {time.perf_counter() - t:.2f} s",
                  file=_sys.stderr, flush=True)

    for w in range(args.warmup):
        tw = time.perf_counter()
        wave(10_000 + w)
        progress("warmup", w, args.warmup, tw)
    dist.barrier()
    if device.type == "cuda":
        torch.cuda.synchronize(device)
    t0 = time.perf_counter()
    toks, lats = 0, []
    if rank == 0:
        eng.head.host_s, eng.head.ticks = 0.0, 0
        eng.head.host_by_kind = {k: [0.0, 0] for k in eng.head.host_by_kind}
        eng.head.phase_s = {k: 0.0 for k in eng.head.phase_s}
    for s in range(args.steps):
        tw = time.perf_counter()
        n, l = wave(s)
        toks += n
        lats += l
        progress("timed", s, args.steps, tw)
    if device.type == "cuda":
        torch.cuda.synchronize(device)
    dist.barrier()
    dt = torch.tensor([time.perf_counter() - t0], dtype=torch.float64,
                      device=device if dist.get_backend() == "nccl" else "cpu")
    dist.all_reduce(dt, op=dist.ReduceOp.MAX)
    from .transport import gather_rank_info
    infos = gather_rank_info(device)
    eng.shutdown() if rank == 0 else eng.serve()
    dist.barrier()
    eng.channel.close()
    dist.destroy_process_group()
    if rank != 0:
        return None
    snap = eng.head.stats.snapshot()
    snap["head_host_ms_per_tick"] = round(1e3 * eng.head.host_s / max(1, eng.head.ticks), 4)
    hd = eng.head.host_by_kind[DECODE]
    snap["head_host_ms_per_decode_tick"] = round(1e3 * hd[0] / max(1, hd[1]), 4)
    snap["head_phase_ms_per_tick"] = {k: round(1e3 * v / max(1, eng.head.ticks), 4)
                                      for k, v in eng.head.phase_s.items()}
    snap["control_plane"] = eng.channel.ctrl_kind
    return {"tokens": toks, "seconds": float(dt.item()), "latencies": lats,
            "global_batch": per_wave, "parallelism": f"pp{world}", "engine": snap,
            "data_plane": eng.channel.data_plane, "ranks_info": infos}


def run_one_session(eng: DistributedPipelineEngine):
    """Serve exactly one head session on a non-head rank (bench lockstep)."""
    serve_session(eng.stage, eng.channel)
