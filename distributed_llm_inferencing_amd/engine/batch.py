"""Per-step batch metadata shared by the scheduler, the model and the pipeline transport.

A step is all-prefill (packed prompts, causal varlen attention over the prompt), all-decode
(one token per running sequence, paged attention over the cache) or mixed (a prefill step
whose first ``num_decode`` sequences are one-token decode rows of running sequences). The host
builds the metadata once per step as ONE packed int32 buffer (``pack``/``unpack``) so it
can travel with the activations between pipeline stages in a single message, and be
copied into static device buffers for hipGraph replay.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional

import numpy as np
import torch

PREFILL, DECODE, EMPTY, STOP = 1, 2, 0, 3
HEADER_LEN = 16


@dataclass
class StepMeta:
    """Host-side description of one step (plain Python / numpy)."""
    kind: int
    seq_ids: List[int] = field(default_factory=list)       # engine slot ids, one per sequence
    input_ids: Optional[np.ndarray] = None                  # [T] int32 (head stage only)
    positions: Optional[np.ndarray] = None                  # [T] int32
    slot_mapping: Optional[np.ndarray] = None               # [T] int32
    seq_lens: Optional[np.ndarray] = None                   # [S] prefill: prompt lens
    context_lens: Optional[np.ndarray] = None               # [S] decode: ctx incl. new token
    block_tables: Optional[np.ndarray] = None               # [S, max_blocks] int32
    temperature: Optional[np.ndarray] = None                # [S] float32
    top_k: Optional[np.ndarray] = None                      # [S] int32
    top_p: Optional[np.ndarray] = None                      # [S] float32
    seeds: Optional[np.ndarray] = None                      # [S] int64
    microbatch: int = 0
    step_id: int = 0
    # lookahead (single stage, not on the wire): row of the in-flight step's device output
    # that holds this sequence's input id, -1 = input_ids holds it
    feed_src: Optional[np.ndarray] = None
    # chunked prefill (not on the wire): True for rows whose chunk completes the prompt; the
    # token sampled for any other row is discarded. None = every row samples.
    sample_mask: Optional[np.ndarray] = None
    # mixed step (header word 9 on the wire): the first num_decode sequences are decode
    # rows (one token each, attended by the decode kernel), the rest prefill chunks
    num_decode: int = 0
    # columns of block_tables that hold blocks (the scheduler knows it; pack trims to it)
    table_used: Optional[int] = None
    # seq_ids as int64 numpy (set by the decode scheduler; saves list -> array conversions)
    seq_ids_arr: Optional[np.ndarray] = None
    # the payload already packed by the C++ scheduler core (decode fast path), its
    # un-trimmed table width, and the core's identity for the matching update
    packed_payload: Optional[np.ndarray] = None
    table_width_full: int = 0
    core: Optional[tuple] = None

    @property
    def num_seqs(self) -> int:
        return len(self.seq_ids)

    @property
    def num_sampled(self) -> int:
        return self.num_seqs if self.sample_mask is None else int(self.sample_mask.sum())

    @property
    def num_tokens(self) -> int:
        return 0 if self.positions is None else int(self.positions.shape[0])

    # ---- wire format: header (int64) + payload (int32) ------------------------------------
    def pack(self) -> (np.ndarray, np.ndarray):
        S, T = self.num_seqs, self.num_tokens
        if self.packed_payload is not None:
            header = np.zeros(HEADER_LEN, dtype=np.int64)
            header[:7] = [self.kind, S, T, int(self.table_used), self.packed_payload.shape[0],
                          self.microbatch, self.step_id]
            header[7] = 1
            header[8] = max(int(self.table_width_full), int(self.table_used))
            header[9] = int(self.num_decode)
            return header, self.packed_payload
        tables = self.block_tables
        width = 0 if tables is None else int(tables.shape[1])
        if tables is not None and tables.shape[1] > 1:
            # trailing all-zero columns are dropped and restored by unpack (zeros either way:
            # padding or block 0): a 100-token decode needs 7 of the 32 columns, 2.5x less
            # control-plane payload
            if self.table_used is not None:
                keep = int(self.table_used)
            else:
                used = np.flatnonzero(np.asarray(tables).any(axis=0))
                keep = int(used[-1]) + 1 if used.size else 1
            if keep < tables.shape[1]:
                tables = tables[:, :keep]
        mb = 0 if tables is None else int(tables.shape[1])
        n = S + 3 * T + 2 * S + S * mb + 3 * S + 2 * S
        payload = np.empty(n, dtype=np.int32)
        o = 0

        def put(a, cnt, f32=False):
            nonlocal o
            if a is None:
                payload[o:o + cnt] = 0
            elif f32:
                payload[o:o + cnt] = np.asarray(a, dtype=np.float32).reshape(-1).view(np.int32)
            else:
                payload[o:o + cnt].reshape(np.shape(a) if np.ndim(a) > 1 else -1)[...] = a
            o += cnt
        put(self.seq_ids_arr if self.seq_ids_arr is not None else
            np.asarray(self.seq_ids, dtype=np.int64), S)
        put(self.input_ids, T)
        put(self.positions, T)
        put(self.slot_mapping, T)
        put(self.seq_lens, S)
        put(self.context_lens, S)
        put(tables, S * mb)
        put(self.temperature, S, f32=True)
        put(self.top_k, S)
        put(self.top_p, S, f32=True)
        if self.seeds is None:
            payload[o:o + 2 * S] = 0
        else:
            payload[o:o + 2 * S] = np.asarray(self.seeds, dtype=np.int64).view(np.int32)
        o += 2 * S
        header = np.zeros(HEADER_LEN, dtype=np.int64)
        header[:7] = [self.kind, S, T, mb, payload.shape[0], self.microbatch, self.step_id]
        header[7] = 1 if self.input_ids is not None else 0
        header[8] = width
        header[9] = int(self.num_decode)          # mixed step: leading one-token decode rows
        return header, payload

    @staticmethod
    def unpack(header: np.ndarray, payload: np.ndarray) -> "StepMeta":
        kind, S, T, mb, _n, micro, step = (int(v) for v in header[:7])
        o = 0

        def take(n, dt=np.int32):
            nonlocal o
            a = payload[o:o + n]
            o += n
            return a.view(dt).copy() if dt != np.int32 else a.copy()

        seq_ids = take(S).tolist()
        input_ids = take(T)
        positions, slots = take(T), take(T)
        seq_lens, ctx = take(S), take(S)
        bt = take(S * mb).reshape(S, mb)
        width = int(header[8])
        if width > mb:                       # restore the trimmed all-zero columns
            bt = np.concatenate([bt, np.zeros((S, width - mb), np.int32)], axis=1)
        temp = take(S, np.float32)
        topk = take(S)
        topp = take(S, np.float32)
        seeds = take(2 * S).view(np.int64).copy()
        return StepMeta(kind=kind, seq_ids=seq_ids,
                        input_ids=input_ids if header[7] else None, positions=positions,
                        slot_mapping=slots, seq_lens=seq_lens, context_lens=ctx,
                        block_tables=bt, temperature=temp, top_k=topk, top_p=topp, seeds=seeds,
                        microbatch=micro, step_id=step, num_decode=int(header[9]))


def _i32(a, n):
    if a is None:
        return np.zeros(n, dtype=np.int32)
    return np.ascontiguousarray(a, dtype=np.int32).reshape(-1)


def _f32_as_i32(a, n):
    if a is None:
        return np.zeros(n, dtype=np.int32)
    return np.ascontiguousarray(a, dtype=np.float32).reshape(-1).view(np.int32)


@dataclass
class DeviceBatch:
    """Device tensors for one step (what the model consumes)."""
    kind: int
    num_seqs: int
    num_tokens: int
    input_ids: Optional[torch.Tensor]
    positions: torch.Tensor
    slot_mapping: torch.Tensor
    cu_seqlens: Optional[torch.Tensor] = None
    max_seqlen: int = 0
    last_token_idx: Optional[torch.Tensor] = None
    block_tables: Optional[torch.Tensor] = None
    context_lens: Optional[torch.Tensor] = None
    max_context: int = 0
    temperature: Optional[torch.Tensor] = None
    top_k: Optional[torch.Tensor] = None
    top_p: Optional[torch.Tensor] = None
    seeds: Optional[torch.Tensor] = None
    # mixed step: decode rows [0, num_decode) (their max context = max_context_decode) and the
    # prefill part's own cu_seqlens / max_seqlen over rows [num_decode, T)
    num_decode: int = 0
    max_context_decode: int = 0
    cu_seqlens_prefill: Optional[torch.Tensor] = None
    max_seqlen_prefill: int = 0

    @property
    def is_prefill(self) -> bool:
        return self.kind == PREFILL


def to_device(meta: StepMeta, device, pin: bool = True) -> DeviceBatch:
    """Every per-step array packed into ONE int32 host buffer (pinned on GPU), ONE H2D copy,
    then device-side views: an eager prefill / mixed step pays a single transfer."""
    dev = torch.device(device)
    S, T = meta.num_seqs, meta.num_tokens
    parts: list = []             # (name, int32 words, dtype, shape)
    nwords = [0]

    def add(name, a, dt):
        if a is None:
            return
        a = np.ascontiguousarray(a)
        if dt == torch.int64:
            a = a.astype(np.int64, copy=False)
            nwords[0] += nwords[0] & 1                   # 8-byte aligned
        elif dt == torch.float32:
            a = a.astype(np.float32, copy=False)
        else:
            a = a.astype(np.int32, copy=False)
        w = a.reshape(-1).view(np.int32)
        parts.append((name, nwords[0], w, dt, a.shape))
        nwords[0] += w.shape[0]

    add("input_ids", meta.input_ids, torch.int32)
    add("positions", meta.positions, torch.int32)
    add("slot_mapping", meta.slot_mapping, torch.int32)
    add("temperature", meta.temperature, torch.float32)
    add("top_k", meta.top_k, torch.int32)
    add("top_p", meta.top_p, torch.float32)
    add("seeds", meta.seeds, torch.int64)
    nd = int(meta.num_decode) if meta.kind == PREFILL else 0
    paged = False
    if meta.kind == PREFILL:
        lens = np.asarray(meta.seq_lens, dtype=np.int64)
        cu = np.zeros(S + 1, dtype=np.int32)
        cu[1:] = np.cumsum(lens)
        add("cu_seqlens", cu, torch.int32)
        add("last_token_idx", cu[1:] - 1, torch.int64)
        paged = meta.block_tables is not None and np.shape(meta.block_tables)[1] > 0
        if nd:
            add("cu_seqlens_prefill", cu[nd:] - nd, torch.int32)
    if meta.kind != PREFILL or paged:
        add("block_tables", meta.block_tables, torch.int32)
        add("context_lens", meta.context_lens, torch.int32)
    buf = np.empty(max(1, nwords[0]), dtype=np.int32)
    for _, o, w, _, _ in parts:
        buf[o:o + w.shape[0]] = w
    host = torch.from_numpy(buf)
    if dev.type == "cuda":
        if pin:
            pinned = torch.empty(buf.shape, dtype=torch.int32, pin_memory=True)
            pinned.numpy()[:] = buf
            host = pinned
        packed = host.to(dev, non_blocking=True)
    else:
        packed = host
    v = {}
    for name, o, w, dt, shape in parts:
        x = packed[o:o + w.shape[0]]
        if dt != torch.int32:
            x = x.view(dt)
        v[name] = x.view(shape) if len(shape) > 1 else x
    db = DeviceBatch(kind=meta.kind, num_seqs=S, num_tokens=T,
                     input_ids=v.get("input_ids"), positions=v.get("positions"),
                     slot_mapping=v.get("slot_mapping"), temperature=v.get("temperature"),
                     top_k=v.get("top_k"), top_p=v.get("top_p"), seeds=v.get("seeds"))
    if meta.kind == PREFILL:
        db.cu_seqlens = v["cu_seqlens"]
        db.max_seqlen = int(lens.max()) if S else 0
        db.last_token_idx = v["last_token_idx"]
        if paged:
            # chunked prefill: queries attend over the paged cache (earlier chunks + this one)
            db.block_tables = v["block_tables"]
            db.context_lens = v["context_lens"]
            db.max_context = int(np.max(meta.context_lens)) if S else 0
        if nd:
            ctx = np.asarray(meta.context_lens)
            db.num_decode = nd
            db.max_context_decode = int(ctx[:nd].max())
            db.cu_seqlens_prefill = v["cu_seqlens_prefill"]
            db.max_seqlen_prefill = int(lens[nd:].max()) if S > nd else 0
    else:
        db.block_tables = v.get("block_tables")
        db.context_lens = v.get("context_lens")
        db.max_context = int(np.max(meta.context_lens)) if S else 0
    return db
