"""Continuous-batching scheduler (iteration-level, prefill-first), microbatch aware.

Replaces the reference's one-request-at-a-time worker (1 sync gunicorn worker,
``worker/Dockerfile:45``; batch = 1): every engine step either admits a packed batch of
waiting prompts (prefill) or advances every running sequence of one microbatch by one
token (decode). With pipeline parallelism the running set is split into M microbatches
(M = number of stages) that circulate through the pipeline; each microbatch is scheduled
only after its previous step's tokens came back.

KV memory comes from the C++ ``BlockManager``; when a decode step cannot get a block the
newest sequence of that microbatch is preempted (its blocks freed, re-queued at the front,
recomputed later from prompt + generated tokens).
"""
from __future__ import annotations

import time
import zlib
from collections import deque
from typing import Dict, List, Optional

import numpy as np

from ..runtime import BlockManager
from .batch import DECODE, PREFILL, StepMeta
from .sequence import SamplingParams, Sequence, SeqState, row_seed


class Scheduler:
    def __init__(self, block_manager: BlockManager, max_seqs_per_mb: int = 256,
                 max_prefill_tokens: int = 16384, num_microbatches: int = 1,
                 eos_token_id: Optional[int] = None, max_model_len: int = 4096,
                 table_width: Optional[int] = None):
        self.bm = block_manager
        self.bs = block_manager.block_size
        self.max_seqs = max_seqs_per_mb
        self.max_prefill_tokens = max_prefill_tokens
        self.M = num_microbatches
        self.eos = eos_token_id
        self.max_model_len = max_model_len
        # fixed block-table width (static for hipGraph replay) = blocks for max_model_len
        self.table_width = table_width or -(-max_model_len // self.bs)
        self.waiting: deque = deque()
        self.running: List[List[Sequence]] = [[] for _ in range(self.M)]
        self.seqs: Dict[int, Sequence] = {}
        self.finished: List[Sequence] = []
        self._next_id = 0
        self._step = 0

    # ------------------------------------------------------------------ requests
    def add_request(self, request_id: str, prompt_ids: List[int],
                    params: Optional[SamplingParams] = None) -> Sequence:
        params = params or SamplingParams()
        if len(prompt_ids) == 0:
            raise ValueError("empty prompt")
        if len(prompt_ids) >= self.max_model_len:
            raise ValueError(f"prompt of {len(prompt_ids)} tokens exceeds max_model_len "
                             f"{self.max_model_len}")
        sid = self._next_id
        self._next_id += 1
        seed = (params.seed if params.seed is not None
                else zlib.crc32(f"{request_id}:{sid}".encode()) & 0x7FFFFFFF)
        seq = Sequence(seq_id=sid, request_id=request_id, prompt_ids=list(prompt_ids),
                       params=params, seed=int(seed))
        self.seqs[sid] = seq
        if params.budget(len(prompt_ids)) <= 0:
            self._finish(seq, "length")
        else:
            self.waiting.append(seq)
        return seq

    def abort(self, request_id: str) -> bool:
        for seq in list(self.seqs.values()):
            if seq.request_id == request_id and seq.state != SeqState.FINISHED:
                self._finish(seq, "abort")
                return True
        return False

    def has_work(self) -> bool:
        return bool(self.waiting) or any(self.running)

    def num_running(self) -> int:
        return sum(len(r) for r in self.running)

    # ------------------------------------------------------------------ internals
    def _finish(self, seq: Sequence, reason: str):
        if seq.state == SeqState.FINISHED:
            return
        seq.state = SeqState.FINISHED
        seq.finish_reason = reason
        seq.finish_time = time.perf_counter()
        self.bm.free(seq.seq_id)
        if seq in self.waiting:
            self.waiting.remove(seq)
        for r in self.running:
            if seq in r:
                r.remove(seq)
        self.finished.append(seq)

    def _expire(self):
        now = time.perf_counter()
        for seq in list(self.waiting) + [s for r in self.running for s in r]:
            dl = seq.deadline
            if dl is not None and now > dl:
                self._finish(seq, "timeout")

    def _preempt(self, mb: int) -> bool:
        r = self.running[mb]
        if not r:
            return False
        victim = max(r, key=lambda s: s.arrival)
        r.remove(victim)
        self.bm.free(victim.seq_id)
        victim.state = SeqState.WAITING
        victim.num_preemptions += 1
        self.waiting.appendleft(victim)
        return True

    def _sampling_arrays(self, seqs: List[Sequence]):
        n = len(seqs)
        temp = np.empty(n, np.float32)
        topk = np.empty(n, np.int32)
        topp = np.empty(n, np.float32)
        seeds = np.empty(n, np.int64)
        for i, s in enumerate(seqs):
            p = s.params
            temp[i] = p.effective_temperature()
            topk[i] = p.top_k
            topp[i] = p.top_p
            seeds[i] = row_seed(s.seed, len(s.output_ids))
        return temp, topk, topp, seeds

    # ------------------------------------------------------------------ scheduling
    def schedule(self, mb: int = 0) -> Optional[StepMeta]:
        """Next step for microbatch ``mb`` (None if it has nothing to do)."""
        self._expire()
        self._step += 1
        meta = self._try_prefill(mb)
        if meta is not None:
            return meta
        return self._decode(mb)

    def _least_loaded_ok(self, mb: int) -> bool:
        # balance admissions across microbatches: only admit into mb if it is among the least loaded
        loads = [len(r) for r in self.running]
        return len(self.running[mb]) <= min(loads)

    def _try_prefill(self, mb: int) -> Optional[StepMeta]:
        if not self.waiting or (self.M > 1 and not self._least_loaded_ok(mb)):
            return None
        picked: List[Sequence] = []
        tokens = 0
        room = self.max_seqs - len(self.running[mb])
        while self.waiting and len(picked) < room:
            seq = self.waiting[0]
            n = seq.total_len
            if picked and tokens + n > self.max_prefill_tokens:
                break
            if not self.bm.ensure(seq.seq_id, n):
                break
            self.waiting.popleft()
            picked.append(seq)
            tokens += n
        if not picked:
            return None
        for s in picked:
            s.state = SeqState.RUNNING
            s.microbatch = mb
            self.running[mb].append(s)
        lens = np.array([s.total_len for s in picked], dtype=np.int32)
        ids = np.concatenate([np.asarray(s.all_ids(), dtype=np.int32) for s in picked])
        pos = np.concatenate([np.arange(n, dtype=np.int32) for n in lens])
        sid = [s.seq_id for s in picked]
        slots = self.bm.slot_mapping(sid, np.zeros(len(picked), np.int32), lens)
        temp, topk, topp, seeds = self._sampling_arrays(picked)
        return StepMeta(kind=PREFILL, seq_ids=sid, input_ids=ids, positions=pos,
                        slot_mapping=slots, seq_lens=lens, context_lens=lens.copy(),
                        block_tables=np.zeros((len(picked), 0), np.int32), temperature=temp,
                        top_k=topk, top_p=topp, seeds=seeds, microbatch=mb, step_id=self._step)

    def _decode(self, mb: int) -> Optional[StepMeta]:
        r = self.running[mb]
        i = 0
        while i < len(r):
            seq = r[i]
            if not self.bm.ensure(seq.seq_id, seq.total_len):
                if not self._preempt(mb):
                    break
                continue           # list changed; re-check same index
            i += 1
        seqs = list(r)
        if not seqs:
            return None
        ctx = np.array([s.total_len for s in seqs], dtype=np.int32)
        sid = [s.seq_id for s in seqs]
        last = np.array([s.output_ids[-1] if s.output_ids else s.prompt_ids[-1] for s in seqs],
                        dtype=np.int32)
        slots = self.bm.slot_mapping(sid, ctx - 1, np.ones(len(seqs), np.int32))
        tables = self.bm.fill_tables(sid, self.table_width)
        temp, topk, topp, seeds = self._sampling_arrays(seqs)
        return StepMeta(kind=DECODE, seq_ids=sid, input_ids=last, positions=ctx - 1,
                        slot_mapping=slots, seq_lens=np.ones(len(seqs), np.int32),
                        context_lens=ctx, block_tables=tables, temperature=temp, top_k=topk,
                        top_p=topp, seeds=seeds, microbatch=mb, step_id=self._step)

    # ------------------------------------------------------------------ results
    def update(self, meta: StepMeta, tokens) -> List[Sequence]:
        """Apply sampled tokens of a finished step; returns sequences that finished."""
        tokens = np.asarray(tokens).reshape(-1)
        done = []
        now = time.perf_counter()
        for i, sid in enumerate(meta.seq_ids):
            seq = self.seqs.get(sid)
            if seq is None or seq.state != SeqState.RUNNING:
                continue
            t = int(tokens[i])
            seq.output_ids.append(t)
            if seq.first_token_time is None:
                seq.first_token_time = now
            p = seq.params
            reason = None
            if len(seq.output_ids) >= p.budget(seq.prompt_len):
                reason = "length"
            elif not p.ignore_eos and self.eos is not None and t == self.eos:
                reason = "stop"
            elif t in p.stop_token_ids:
                reason = "stop"
            elif seq.total_len >= self.max_model_len:
                reason = "length"
            if reason:
                self._finish(seq, reason)
                done.append(seq)
        return done

    def pop_finished(self) -> List[Sequence]:
        out, self.finished = self.finished, []
        for s in out:
            self.seqs.pop(s.seq_id, None)
        return out
