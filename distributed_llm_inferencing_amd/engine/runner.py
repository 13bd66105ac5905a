"""Executes steps of one pipeline stage on its device, with hipGraph-captured decode.

Decode steps have a fixed shape per batch-size bucket, so each bucket's whole stage forward
(all layers, and on the last stage the LM head + sampler) is captured once into a
``torch.cuda.CUDAGraph`` (a hipGraph on ROCm) and replayed: one graph launch per step per
stage instead of ~10 kernel launches per layer. All per-step metadata
lives in ONE static int32 device buffer refreshed by ONE pinned H2D copy before replay.
Padded rows (bucket > live sequences) carry slot = -1 (no KV write) and context 0.

Prefill steps (variable packed length) run eagerly.
"""
from __future__ import annotations

import os
from typing import Dict, Optional

import numpy as np
import torch

from .. import ops
from ..models.model import TransformerLM
from .batch import DECODE, DeviceBatch, StepMeta, to_device
from .kv_cache import KVCache

DEFAULT_BUCKETS = (1, 2, 4, 8, 16, 24, 32, 48, 64, 96, 128, 160, 192, 256, 320, 384, 448, 512)
HOST_RING = 4          # pinned metadata staging buffers per runner


class StageRunner:
    def __init__(self, model: TransformerLM, kv: KVCache, max_batch: int, table_width: int,
                 use_graphs: Optional[bool] = None, buckets=DEFAULT_BUCKETS):
        self.model = model
        self.kv = kv
        self.kv_layers = kv.layers()
        self.device = model.device
        self.max_batch = max_batch
        self.W = table_width
        if use_graphs is None:
            use_graphs = (self.device.type == "cuda" and os.environ.get("DLI_NO_GRAPHS", "0") != "1"
                          and os.environ.get("DLI_DEBUG_SYNC", "0") != "1")
        self.use_graphs = use_graphs
        self.buckets = sorted({b for b in buckets if b < max_batch} | {max_batch})
        self.graphs: Dict[int, torch.cuda.CUDAGraph] = {}
        self.graph_out: Dict[int, torch.Tensor] = {}
        # pipeline data plane captured INTO the decode graphs (set_piped): pre(b) receives
        # the bucket's input rows into hidden_in before the layers, post(b, out) sends the
        # output after them, so a stage's decode tick is one H2D + one graph launch
        self.piped = None
        self.force_eager = False        # lockstep users (EP): run this step's decode eagerly
        self.replays = 0
        self.uploads = 0
        self._pool = None
        self.hidden_in = None
        if self.use_graphs:
            self._init_static()

    # ------------------------------------------------------------------ static buffers
    def _init_static(self):
        B, W = self.max_batch, self.W
        # layout (int32 words):
        #   seeds(2B) | ids | pos | slots | ctx | temp | topk | topp | src | tables(B*W)
        # seeds first: an int64 view needs an even word offset whatever B is (B = 1 put it at
        # word 7); src = lookahead feed rows (StepMeta.feed_src, -1 = host id)
        self._off = {}
        o = 0
        for name, n in (("seeds", 2 * B), ("ids", B), ("pos", B), ("slots", B), ("ctx", B),
                        ("temp", B), ("topk", B), ("topp", B), ("src", B),
                        ("tables", B * W)):
            self._off[name] = (o, n)
            o += n
        self._nwords = o
        self.meta_dev = torch.zeros(o, dtype=torch.int32, device=self.device)
        # a ring of pinned staging buffers: the host fills step k+1's metadata while step
        # k's upload (stream-ordered behind step k's receive on a pipeline stage) is still
        # pending; reusing a buffer waits only for the upload HOST_RING steps back, so a
        # stage host runs up to HOST_RING - 1 ticks ahead of its GPU
        self._ring = [torch.zeros(o, dtype=torch.int32).pin_memory() for _ in range(HOST_RING)]
        self._ring_np = [t.numpy() for t in self._ring]
        self._ring_ev = [torch.cuda.Event() for _ in range(HOST_RING)]
        self._ring_used = [False] * HOST_RING
        self._slot = 0
        self.meta_host = self._ring[0]
        self._host_np = self._ring_np[0]
        self.host_waits = 0                          # fills that found their buffer busy
        self.hidden_in = None
        if not self.model.is_first:
            self.hidden_in = torch.zeros(B, self.model.cfg.hidden_size, dtype=torch.bfloat16,
                                         device=self.device)

    def _view(self, name, b, dtype=torch.int32):
        o, n = self._off[name]
        v = self.meta_dev[o:o + n]
        if dtype == torch.float32:
            v = v.view(torch.float32)
        elif dtype == torch.int64:
            v = v.view(torch.int64)
        if name == "tables":
            return v.view(self.max_batch, self.W)[:b]
        return v[:b]

    def _static_batch(self, b: int) -> DeviceBatch:
        return DeviceBatch(kind=DECODE, num_seqs=b, num_tokens=b,
                           input_ids=self._view("ids", b), positions=self._view("pos", b),
                           slot_mapping=self._view("slots", b),
                           block_tables=self._view("tables", b),
                           context_lens=self._view("ctx", b),
                           max_context=self.W * self.kv.block_size,
                           temperature=self._view("temp", b, torch.float32),
                           top_k=self._view("topk", b), top_p=self._view("topp", b, torch.float32),
                           seeds=self._view("seeds", b, torch.int64))

    def _fill_host(self, meta: StepMeta, b: int):
        j = self._slot = (self._slot + 1) % HOST_RING
        if self._ring_used[j]:
            ev = self._ring_ev[j]
            if not ev.query():                       # its H2D (HOST_RING steps back) pending
                self.host_waits += 1
                ev.synchronize()
        self.meta_host, self._host_np = self._ring[j], self._ring_np[j]
        h = self._host_np
        S = meta.num_seqs

        def put(name, arr, pad):
            o, _ = self._off[name]
            a = np.ascontiguousarray(arr).reshape(-1)
            if a.dtype != np.int32:
                a = a.view(np.int32)
            h[o:o + a.shape[0]] = a
            extra = (b - S) * (2 if name == "seeds" else 1)
            if extra > 0:
                h[o + a.shape[0]:o + a.shape[0] + extra] = pad
        put("ids", meta.input_ids if meta.input_ids is not None else np.zeros(S, np.int32), 0)
        put("pos", meta.positions, 0)
        put("slots", meta.slot_mapping, -1)
        put("ctx", meta.context_lens, 0)
        put("temp", meta.temperature.astype(np.float32), 0)
        put("topk", meta.top_k, 1)
        put("topp", meta.top_p.astype(np.float32), np.float32(1.0).view(np.int32))
        put("seeds", meta.seeds.astype(np.int64), 0)
        put("src", meta.feed_src if meta.feed_src is not None else np.full(S, -1, np.int32), -1)
        o, _ = self._off["tables"]
        tb = np.asarray(meta.block_tables, dtype=np.int32)
        if tb.shape[1] != self.W:
            t2 = np.zeros((S, self.W), np.int32)
            t2[:, :min(self.W, tb.shape[1])] = tb[:, :self.W]
            tb = t2
        h[o:o + S * self.W] = tb.reshape(-1)
        if b > S:
            h[o + S * self.W:o + b * self.W] = 0

    def _upload(self, b: int):
        # tables occupy the tail; copy everything up to the last used table row
        o, _ = self._off["tables"]
        n = o + b * self.W
        self.meta_dev[:n].copy_(self.meta_host[:n], non_blocking=True)
        self.uploads += 1
        self._ring_ev[self._slot].record()
        self._ring_used[self._slot] = True

    def _bucket(self, S: int) -> int:
        for b in self.buckets:
            if b >= S:
                return b
        raise ValueError(f"decode batch {S} exceeds max_batch {self.max_batch}")

    def set_piped(self, pre, post) -> None:
        """Capture ``pre(b)`` / ``post(b, out)`` (stream-ordered transport calls, e.g. the
        IPC mailboxes) into every decode graph; graphs captured before are dropped."""
        self.piped = (pre, post)
        self.graphs.clear()
        self.graph_out.clear()

    # ------------------------------------------------------------------ capture
    def _forward_static(self, b: int):
        db = self._static_batch(b)
        hidden = self.hidden_in[:b] if self.hidden_in is not None else None
        return self.model.forward(db, self.kv_layers, hidden=hidden)

    def gemm_shapes(self, M: int):
        """(shapes, weights) of every projection GEMM a decode step of M rows runs here."""
        from ..ops import gemm as G
        m = self.model
        shapes, weights = [], {}
        lp = m.layers[0] if m.layers else {}

        def add(w, epi, rows=M):
            if w is None or w.dim() != 2:
                return
            shapes.append((rows, w.shape[0], w.shape[1], epi))
            weights[(w.shape[0], w.shape[1])] = w
        if m.cfg.arch == "gpt2":
            add(lp.get("wqkv"), "bias"), add(lp.get("wo"), "bias")
            add(lp.get("w_fc"), "bias_gelu"), add(lp.get("w_proj"), "bias")
        else:   # llama family: these feed the fused split-K reduces (ops.linear_*)
            add(lp.get("wqkv"), "splitk"), add(lp.get("wo"), "splitk")
            if not m.cfg.is_moe:
                add(lp.get("w_gu"), "silu_mul"), add(lp.get("w_down"), "splitk")
            # batch-1 / tiny steps: O and down add into the residual in their own epilogue
            # (models/model.py deferred norm) — timed as that op
            if (M <= G.GEMV_MAX_M and G.DEFER_NORM and not m.cfg.is_moe
                    and m.tp_reduce is None):
                add(lp.get("wo"), "res"), add(lp.get("w_down"), "res")
        if m.is_last and not m.vocab_parallel:
            head = m.params["embed"] if m.cfg.tie_embeddings else m.params.get("lm_head")
            add(head, ops.HEAD_EPI)
        if m.vocab_parallel:                 # this rank's slice of the LM head
            add(m.params.get("head_slice"), ops.HEAD_EPI)
        return shapes, weights

    def tune_lock(self):
        """Ranks that share one GPU (same-device rehearsals: DLI_SAME_DEVICE=1) time their
        GEMM candidates one process at a time: tuned concurrently, each plan was measured
        under the other ranks' load and the pins came out at random (an expert-parallel rank
        ran 947 us grouped GEMMs that take ~120 us alone). Engines that exchange data during
        capture tune every bucket first, then barrier, then capture (no peer waits on a
        tuning rank inside a bounded device wait)."""
        import contextlib
        if os.environ.get("DLI_SAME_DEVICE", "0") != "1" or self.device.type != "cuda":
            return contextlib.nullcontext()

        @contextlib.contextmanager
        def held():
            import fcntl
            path = f"/tmp/dli_tune_{os.getuid()}_{self.device.index or 0}.lock"
            with open(path, "w") as f:
                fcntl.flock(f, fcntl.LOCK_EX)
                try:
                    torch.cuda.synchronize(self.device)
                    yield
                finally:
                    fcntl.flock(f, fcntl.LOCK_UN)
        return held()

    def autotune(self, buckets=None):
        with self.tune_lock():
            self._autotune(buckets)

    def _autotune(self, buckets=None):
        from ..ops import gemm as G
        log = None
        if os.environ.get("DLI_GEMM_AUTOTUNE_LOG", "0") == "1":
            import sys
            log = lambda m: print(m, file=sys.stderr, flush=True)  # noqa: E731
        m = self.model
        moe = (m.cfg.is_moe and m.layers and m.layers[0].get("w_gu") is not None
               and m.layers[0]["w_gu"].dim() == 3)
        for b in (buckets or self.buckets):
            shapes, weights = self.gemm_shapes(b)
            c = m.cfg
            qkv = ((c.num_heads, c.num_kv_heads, c.head_dim) if c.arch != "gpt2" else None)
            normed = ()
            if (b <= G.GEMV_MAX_M and G.DEFER_NORM and not c.is_moe and c.arch != "gpt2"
                    and m.tp_reduce is None and m.layers):
                lp = m.layers[0]           # batch-1 QKV and gate/up read a deferred norm
                normed = {(lp["wqkv"].shape[0], lp["wqkv"].shape[1], "splitk"),
                          (lp["w_gu"].shape[0], lp["w_gu"].shape[1], "silu_mul")}
            G.autotune(shapes, weights, self.device, log=log, qkv_heads=qkv, normed_in=normed)
            if moe:      # grouped expert GEMMs: rows = b tokens x top-k (uniform routing)
                lp = m.layers[0]
                rows = b * m.cfg.top_k_experts
                G.autotune_grouped(rows, lp["w_gu"], "silu_mul", log=log)
                G.autotune_grouped(rows, lp["w_down"], "none", log=log)

    def autotune_prefill(self, max_tokens: int) -> None:
        """GEMM plans of prefill steps, one per power-of-two token bucket from 2048 up to the
        bucket of ``max_tokens``: our 8-phase kernel against our 4-wave kernel, the faster pinned
        (``ops.gemm.prefill_candidates``). Skipped like the decode autotune
        (DLI_GEMM_AUTOTUNE=0, non-GPU) and by DLI_TUNE_PREFILL=0."""
        if (os.environ.get("DLI_GEMM_AUTOTUNE", "1") != "1" or self.device.type != "cuda"
                or os.environ.get("DLI_TUNE_PREFILL", "1") != "1"):
            return
        from ..ops import gemm as G
        log = None
        if os.environ.get("DLI_GEMM_AUTOTUNE_LOG", "0") == "1":
            import sys
            log = lambda m: print(m, file=sys.stderr, flush=True)  # noqa: E731
        top = G._bucket(max(max_tokens, 2048))
        c = self.model.cfg
        qkv = (c.num_heads, c.num_kv_heads, c.head_dim) if c.arch != "gpt2" else None
        b = 2048
        with self.tune_lock():
            while b <= top:
                shapes, weights = self.gemm_shapes(b)
                shapes = [s for s in shapes if s[3] != "f32"]     # prefill's LM head: last rows
                G.autotune(shapes, weights, self.device, iters=3, log=log, cold_bytes=1,
                           qkv_heads=qkv, candidates=G.prefill_candidates)
                b *= 2

    def autotune_mixed(self, max_rows: int) -> None:
        """GEMM plans for mixed prefill+decode steps (a running batch's decode rows plus the
        prompt tokens admitted with them: 512 < M <= 1024 for a full 512-row batch). They run
        eagerly, and without these buckets their GEMMs took the fitted heuristic's 128-row
        tiles, not the tuned decode plans."""
        if os.environ.get("DLI_GEMM_AUTOTUNE", "1") != "1" or self.device.type != "cuda":
            return
        top = min(1024, max_rows)
        buckets = [m for m in range(640, top + 128, 128) if m > self.max_batch and m <= 1024]
        if buckets:
            self.autotune(buckets)

    def capture(self, buckets=None):
        """Warm up and capture decode graphs for the given buckets (default: all)."""
        if not self.use_graphs:
            return
        # Measured in-situ on MI355X (Llama-3-8B decode): cold-weight autotune at capture is
        # +2.6 % at batch 512 and +12 % at batch 256 over the fitted heuristic, for ~5 s of
        # startup (profiles/r1_final/autotune_ab.txt). DLI_GEMM_AUTOTUNE=0 turns it off.
        if os.environ.get("DLI_GEMM_AUTOTUNE", "1") == "1":
            self.autotune(buckets)
        for b in (buckets or self.buckets):
            if b in self.graphs:
                continue
            # warmup: all rows padded (slot -1, ctx 0) -> no cache writes, no attention reads
            torch.cuda.synchronize(self.device)      # no staged upload still reads the buffer
            h = self._host_np
            h[:] = 0
            for name, pad in (("slots", -1), ("topk", 1)):
                o, n = self._off[name]
                h[o:o + n] = pad
            self.meta_dev.copy_(self.meta_host)
            s = torch.cuda.Stream(self.device)
            s.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(s):
                for _ in range(2):
                    self._forward_static(b)
            torch.cuda.current_stream(self.device).wait_stream(s)
            torch.cuda.synchronize(self.device)
            g = torch.cuda.CUDAGraph()
            # thread-local capture: the RCCL process group's watchdog thread keeps polling
            # its events while a stage captures; under the default global mode such a call
            # from another thread invalidates the capture (and aborts the watchdog)
            with torch.cuda.graph(g, pool=self._pool, capture_error_mode="thread_local"):
                if self.piped is not None and self.piped[0] is not None:
                    self.piped[0](b)
                out = self._forward_static(b)
                if self.piped is not None and self.piped[1] is not None:
                    self.piped[1](b, out)
            if self._pool is None:
                self._pool = g.pool()
            self.graphs[b] = g
            self.graph_out[b] = out
        torch.cuda.synchronize(self.device)

    # ------------------------------------------------------------------ execution
    def input_buffer(self, meta: StepMeta) -> Optional[torch.Tensor]:
        """Where a pipeline receive can put this step's hidden input so the graph reads it
        in place: the static graph input for captured decode steps (None otherwise)."""
        if (self.use_graphs and self.hidden_in is not None and meta.kind == DECODE
                and meta.num_seqs <= self.max_batch):
            return self.hidden_in[:meta.num_seqs]
        return None

    @staticmethod
    def _feed(ids: torch.Tensor, src: torch.Tensor, feed: torch.Tensor) -> None:
        """Lookahead: ids[i] = feed[src[i]] where src[i] >= 0 (stream-ordered after the step
        that produced ``feed``, before this step's replay overwrites it)."""
        ops.feed_ids(ids, src, feed)

    def run(self, meta: StepMeta, hidden: Optional[torch.Tensor] = None,
            feed: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Returns int32 tokens [S] on the last stage, else the hidden state [T, D].
        ``feed``: the in-flight step's token output, read where ``meta.feed_src`` says."""
        if meta.feed_src is not None and feed is None:
            raise ValueError("step has lookahead rows but no in-flight output to feed them")
        if (meta.kind == DECODE and self.use_graphs and meta.num_seqs <= self.max_batch
                and not self.force_eager):
            S = meta.num_seqs
            b = self._bucket(S)
            if b not in self.graphs:
                self.capture([b])
            self._fill_host(meta, b)
            self._upload(b)
            if meta.feed_src is not None:
                self._feed(self._view("ids", S), self._view("src", S), feed)
            if (self.hidden_in is not None and hidden is not None
                    and hidden.data_ptr() != self.hidden_in.data_ptr()):
                self.hidden_in[:S].copy_(hidden[:S])
            self.graphs[b].replay()
            self.replays += 1
            return self.graph_out[b][:S]
        db = to_device(meta, self.device)
        if meta.feed_src is not None:
            # pinned + non_blocking: a pageable copy would wait for the in-flight step (the
            # one being fed from) and undo the lookahead overlap (mixed steps: 12 ms per step)
            src = torch.from_numpy(np.ascontiguousarray(meta.feed_src, np.int32))
            if self.device.type == "cuda":
                src = src.pin_memory().to(self.device, non_blocking=True)
            self._feed(db.input_ids, src, feed)
        return self.model.forward(db, self.kv_layers, hidden=hidden)
