"""Single-pipeline-stage inference engine (one GPU, or CPU): the worker's model runtime.

Replaces the reference worker's ``model.generate`` call path (``worker/app.py:278-308``,
L1 in SURVEY.md §1) with: C++ paged-KV allocator + continuous-batching scheduler +
hipGraph decode on our HIP kernels. Multi-GPU pipelines use the same pieces through
``parallel/pipeline.py``.
"""
from __future__ import annotations

import itertools
import os
import time
from dataclasses import dataclass, field
from typing import Dict, Iterable, List, Optional, Union

import numpy as np
import torch

from ..models.configs import ModelConfig, get_config
from ..models.model import TransformerLM
from ..runtime import BlockManager
from ..tokenizer import load_tokenizer
from .kv_cache import KVCache, auto_num_blocks
from .runner import StageRunner
from .scheduler import Scheduler
from .sequence import RequestOutput, SamplingParams, Sequence
from ..utils.tracing import SpanLog, StepTimer, trace_range


@dataclass
class EngineStats:
    steps: int = 0
    prefill_steps: int = 0
    decode_steps: int = 0
    tokens_out: int = 0
    prompt_tokens: int = 0
    mixed_steps: int = 0            # prefill steps that also carried decode rows
    busy_s: float = 0.0
    finished: int = 0
    # batch shape per launched step (serving diagnostics): decode rows of decode steps and of
    # mixed steps, prompt tokens of mixed steps, and the scheduler's running / waiting counts
    decode_rows: int = 0
    mixed_decode_rows: int = 0
    running_sum: int = 0
    waiting_sum: int = 0
    latencies: List[float] = field(default_factory=list)

    def snapshot(self) -> dict:
        lat = sorted(self.latencies[-4096:])
        pct = lambda q: lat[min(len(lat) - 1, int(q * len(lat)))] if lat else None  # noqa: E731
        return {"steps": self.steps, "prefill_steps": self.prefill_steps,
                "decode_steps": self.decode_steps, "mixed_steps": self.mixed_steps,
                "output_tokens": self.tokens_out,
                "prompt_tokens": self.prompt_tokens, "finished_requests": self.finished,
                "busy_s": round(self.busy_s, 4),
                "decode_rows": self.decode_rows, "mixed_decode_rows": self.mixed_decode_rows,
                "running_sum": self.running_sum, "waiting_sum": self.waiting_sum,
                "tokens_per_s": (self.tokens_out / self.busy_s) if self.busy_s > 0 else 0.0,
                "p50_latency_s": pct(0.5), "p99_latency_s": pct(0.99)}


class _HostTokens:
    """Sampled ids of a launched step on their way to the host: an async D2H copy into pinned
    memory + event, enqueued right behind the step (before any later replay can overwrite
    the graph's static output buffer)."""

    def __init__(self, tokens: torch.Tensor):
        self.array = None
        if not tokens.is_cuda:
            self.array = tokens.numpy()
            return
        self.host = torch.empty(tokens.shape, dtype=tokens.dtype, pin_memory=True)
        self.host.copy_(tokens, non_blocking=True)
        self.ev = torch.cuda.Event()
        self.ev.record()

    def get(self) -> np.ndarray:
        if self.array is None:
            self.ev.synchronize()
            self.array = self.host.numpy()
        return self.array


def seq_to_output(seq: Sequence, tokenizer=None) -> RequestOutput:
    end = seq.finish_time or time.perf_counter()
    out = RequestOutput(request_id=seq.request_id, prompt_ids=seq.prompt_ids,
                        output_ids=list(seq.output_ids), finish_reason=seq.finish_reason or "",
                        latency_s=end - seq.arrival,
                        ttft_s=(seq.first_token_time - seq.arrival) if seq.first_token_time else None)
    # HF semantics: generate() returns prompt + continuation; the reference decodes
    # outputs[0] (prompt included) with skip_special_tokens=True (worker/app.py:308).
    # Detokenised on first access of ``text``, off the engine's step loop.
    out.tokenizer = tokenizer
    return out


class LLMEngine:
    def __init__(self, model: Union[str, ModelConfig], device: str = "cpu",
                 dtype=torch.bfloat16, max_batch: int = 256, max_model_len: int = 2048,
                 block_size: int = 16, num_blocks: Optional[int] = None,
                 kv_fraction: float = 0.85, seed: int = 0, use_graphs: Optional[bool] = None,
                 params: Optional[Dict[str, torch.Tensor]] = None, tokenizer_path=None,
                 max_prefill_tokens: int = 16384, num_layers: Optional[int] = None,
                 lm: Optional[TransformerLM] = None, lookahead: Optional[bool] = None,
                 max_kv_tokens: Optional[int] = None, mixed_steps: Optional[bool] = None):
        self.cfg = get_config(model, num_layers) if isinstance(model, str) else model
        self.device = torch.device(device)
        if self.device.type == "cuda" and self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        cfg = self.cfg
        if lm is not None:
            self.model = lm
        elif params is None:
            self.model = TransformerLM.random(cfg, device=self.device, dtype=dtype, seed=seed)
        else:
            self.model = TransformerLM(cfg, {k: v.to(self.device) for k, v in params.items()},
                                       device=self.device)
        max_model_len = min(max_model_len, cfg.max_position)
        if num_blocks is None:
            # KV pool sized from free HBM, optionally capped
            num_blocks = auto_num_blocks(cfg, cfg.num_layers, block_size, self.device,
                                         kv_fraction, cap_tokens=max_kv_tokens or 0)
        self.kv = KVCache(cfg, cfg.num_layers, num_blocks, block_size, self.device, dtype)
        self.bm = BlockManager(num_blocks, block_size)
        # mixed prefill+decode steps (DLI_MIXED_STEPS=0 = off); engines in lockstep with peer
        # ranks (EP / TP) pass False so every rank's step kinds stay aligned
        self.mixed_steps = (os.environ.get("DLI_MIXED_STEPS", "1") == "1"
                            if mixed_steps is None else bool(mixed_steps))
        self.scheduler = Scheduler(self.bm, max_seqs_per_mb=max_batch,
                                   max_prefill_tokens=max_prefill_tokens,
                                   eos_token_id=cfg.eos_token_id, max_model_len=max_model_len,
                                   mixed_steps=self.mixed_steps)
        self.runner = StageRunner(self.model, self.kv, max_batch, self.scheduler.table_width,
                                  use_graphs=use_graphs)
        self.tokenizer = load_tokenizer(cfg, tokenizer_path)
        self.stats = EngineStats()
        self.timer = StepTimer()
        self.spans = SpanLog()
        self._ids = itertools.count()
        self.max_batch = max_batch
        self.max_model_len = max_model_len
        # lookahead scheduling (one step in flight ahead of the host); DLI_LOOKAHEAD=0 = off.
        # Engines whose every step must stay in lockstep with peer ranks (EP / TP) pass False.
        self.lookahead = (os.environ.get("DLI_LOOKAHEAD", "1") == "1"
                          if lookahead is None else bool(lookahead))
        self._inflight = None           # (meta, device tokens, host copy) of the in-flight step
        tr = os.environ.get("DLI_STEP_TRACE")
        self._trace = open(tr, "a", buffering=1) if tr else None   # line-buffered: survives a kill

    # ------------------------------------------------------------------ API
    def add_request(self, prompt: Union[str, List[int]], params: Optional[SamplingParams] = None,
                    request_id: Optional[str] = None) -> str:
        rid = request_id or f"req-{next(self._ids)}"
        ids = self.tokenizer.encode(prompt) if isinstance(prompt, str) else list(prompt)
        self.scheduler.add_request(rid, ids, params)
        return rid

    def abort(self, request_id: str) -> bool:
        return self.scheduler.abort(request_id)

    def has_work(self) -> bool:
        return self.scheduler.has_work() or self._inflight is not None

    def warmup(self, buckets=None, serving: bool = False):
        """Capture decode graphs ahead of serving (and touch every GEMM plan), tune the
        prefill GEMM plans (``StageRunner.autotune_prefill``). ``serving``:
        also tune the GEMM plans of mixed prefill+decode steps (requests arriving while a
        batch decodes; a closed benchmark wave has none)."""
        self.runner.capture(buckets)
        self.runner.autotune_prefill(self.scheduler.max_prefill_tokens)
        if serving and self.mixed_steps:
            self.runner.autotune_mixed(self.max_batch + self.scheduler.max_prefill_tokens)

    def step(self) -> List[RequestOutput]:
        """One engine iteration. With lookahead (default) it schedules and launches the next
        step BEFORE the in-flight step's tokens reach the host, then applies those tokens:
        the host's sync, scheduler update and metadata upload overlap the GPU's work instead
        of leaving it idle between steps (measured ~8 % idle at batch 512 without)."""
        t0 = time.perf_counter()
        return self.finish_step(self.plan_step(), t0)

    def plan_step(self):
        """Schedule this iteration's step (against the in-flight one under lookahead);
        None when there is nothing to launch. Lockstep users (expert parallelism) read its
        size before every rank launches."""
        with self.timer.phase("schedule"):
            if not self.scheduler.has_work():
                return None
            prev = self._inflight
            return self.scheduler.schedule(0, inflight=prev[0] if prev else None)

    def finish_step(self, meta, t0: Optional[float] = None) -> List[RequestOutput]:
        """Launch ``meta`` (if any), then apply the tokens of the step that completes now."""
        t0 = time.perf_counter() if t0 is None else t0
        prev = self._inflight
        launched = None
        if meta is not None:
            kind = "prefill" if meta.kind == 1 else "decode"
            with trace_range(f"engine.{kind}[{meta.num_seqs}]"), self.timer.phase(f"run_{kind}"):
                tokens = self.runner.run(meta, feed=prev[1] if prev is not None else None)
            launched = (meta, tokens, _HostTokens(tokens))
            self.stats.steps += 1
            sch = self.scheduler
            self.stats.running_sum += sch.num_running()
            self.stats.waiting_sum += len(sch.waiting)
            if self._trace is not None:         # DLI_STEP_TRACE: one line per launched step
                self._trace.write(f"{time.perf_counter():.6f} {meta.kind} {meta.num_seqs} "
                                  f"{meta.num_decode} {meta.num_tokens} {sch.num_running()} "
                                  f"{len(sch.waiting)}\n")
            if meta.kind == 1:
                self.stats.prefill_steps += 1
                self.stats.prompt_tokens += meta.num_tokens - meta.num_decode
                if meta.num_decode:
                    self.stats.mixed_steps += 1
                    self.stats.mixed_decode_rows += meta.num_decode
            else:
                self.stats.decode_steps += 1
                self.stats.decode_rows += meta.num_seqs
        if self.lookahead:
            self._inflight = launched
            done = prev
        else:
            done = launched
        if done is not None:
            with self.timer.phase("sync"):
                tok = done[2].get()
            with self.timer.phase("update"):
                self.scheduler.update(done[0], tok)
            self.stats.tokens_out += done[0].num_sampled
        if meta is not None or done is not None:
            self.stats.busy_s += time.perf_counter() - t0
        outs = []
        for seq in self.scheduler.pop_finished():
            o = seq_to_output(seq, self.tokenizer)
            self.stats.finished += 1
            self.stats.latencies.append(o.latency_s)
            self.spans.record(o)
            outs.append(o)
        return outs

    def generate(self, prompts: Iterable[Union[str, List[int]]],
                 params: Optional[SamplingParams] = None) -> List[RequestOutput]:
        rids = [self.add_request(p, params) for p in prompts]
        done: Dict[str, RequestOutput] = {}
        while self.has_work():
            for o in self.step():
                done[o.request_id] = o
        for o in self.step():           # flush requests finished at admission
            done[o.request_id] = o
        return [done[r] for r in rids]

    def memory_report(self) -> dict:
        rep = {"weights_bytes": self.model.param_bytes(), "kv_bytes": self.kv.nbytes,
               "kv_capacity_tokens": self.kv.capacity_tokens,
               "num_blocks": self.kv.num_blocks, "free_blocks": self.bm.num_free}
        if self.device.type == "cuda":
            free, total = torch.cuda.mem_get_info(self.device)
            rep.update({"hbm_free": free, "hbm_total": total})
        return rep
