"""Bindings for the host C++ runtime (``lib/libdli_runtime.so``, sources in csrc/runtime):

* ``BlockManager`` — paged-KV block allocator + batched block-table / slot-mapping builders
* ``DecodeCore`` — one microbatch's running sequences + the decode fast path of the
  continuous-batching scheduler (schedule -> packed step metadata, apply sampled tokens)
* ``SafetensorsFile`` — mmap'd safetensors reader with a pinned-staging ring feeding
  ``hipMemcpyAsync`` (GPU) or plain memcpy (CPU); whole tensors or row ranges
* ``ShmRing`` — single-producer / multi-consumer broadcast ring in POSIX shared memory (the
  pipeline's per-tick control plane between the processes of one node)
"""
from __future__ import annotations

import ctypes
import threading
from pathlib import Path
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

LIB_PATH = Path(__file__).resolve().parent.parent / "lib" / "libdli_runtime.so"
_lib = None
_lock = threading.Lock()

_P, _I, _LL = ctypes.c_void_p, ctypes.c_int, ctypes.c_longlong
_SIGS = {
    "dli_bm_create": ([_I, _I], _P),
    "dli_bm_destroy": ([_P], None),
    "dli_bm_num_free": ([_P], _I),
    "dli_bm_num_blocks": ([_P], _I),
    "dli_bm_block_size": ([_P], _I),
    "dli_bm_blocks_needed": ([_P, _LL, _LL], _I),
    "dli_bm_ensure": ([_P, _LL, _LL], _I),
    "dli_bm_free": ([_P, _LL], _I),
    "dli_bm_free_batch": ([_P, _P, _I], _I),
    "dli_bm_table": ([_P, _LL, _P, _I], _I),
    "dli_bm_fill_tables": ([_P, _P, _I, _P, _I], _I),
    "dli_bm_slot_mapping": ([_P, _P, _P, _P, _I, _P], _I),
    "dli_bm_decode_prepare": ([_P, _P, _P, _I, _P, _P, _I], _I),
    "dli_bm_ensure_batch": ([_P, _P, _P, _I], _I),
    "dli_bm_match_prefix": ([_P, _LL, _P, _I], _I),
    "dli_bm_register_prefix": ([_P, _LL, _P, _I, _I], _I),
    "dli_bm_prefix_hits": ([_P], _LL),
    "dli_bm_num_cached": ([_P], _I),
    "dli_mb_create": ([_I, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _I, _I, _I], _P),
    "dli_mb_destroy": ([_P], None),
    "dli_mb_rows": ([_P], _I),
    "dli_mb_steps": ([_P], _I),
    "dli_mb_payload_words": ([_P, _I], _LL),
    "dli_mb_schedule": ([_P, _P, _I, _P, _LL, _P], _LL),
    "dli_mb_update": ([_P, _P, _I, _P, _P], _I),
    "dli_mb_row_history": ([_P, _I, _P], _I),
    "dli_mb_history": ([_P, _P], _I),
    "dli_mb_compact": ([_P, _P, _I], _I),
    "dli_st_open": ([ctypes.c_char_p], _P),
    "dli_st_close": ([_P], None),
    "dli_st_count": ([_P], _I),
    "dli_st_info": ([_P, _I, ctypes.c_char_p, _I, ctypes.c_char_p, _I, _P, _P, _P], _I),
    "dli_st_find": ([_P, ctypes.c_char_p], _I),
    "dli_st_copy_to_host": ([_P, _I, _P], _I),
    "dli_st_load_to_device": ([_P, _P, _P, _I, _P], _LL),
    "dli_st_load_range": ([_P, _I, _LL, _LL, _P, _P, _I], _LL),
    "dli_ring_create": ([ctypes.c_char_p, _LL, _LL, _I], _P),
    "dli_ring_open": ([ctypes.c_char_p, _I], _P),
    "dli_ring_unlink": ([_P], _I),
    "dli_ring_slot_bytes": ([_P], _LL),
    "dli_ring_publish": ([_P, _P, _LL, ctypes.c_double], _I),
    "dli_ring_consume": ([_P, _P, _LL, ctypes.c_double], _LL),
    "dli_ring_peek_len": ([_P, ctypes.c_double], _LL),
    "dli_ring_published": ([_P], _LL),
    "dli_ring_min_consumed": ([_P], _LL),
    "dli_ring_dead": ([_P], _I),
    "dli_ring_close": ([_P], None),
    "dli_ring_destroy": ([_P], None),
    "dli_board_create": ([ctypes.c_char_p, _I], _P),
    "dli_board_open": ([ctypes.c_char_p], _P),
    "dli_board_join": ([_P, _I], _I),
    "dli_board_unlink": ([_P], _I),
    "dli_board_world": ([_P], _I),
    "dli_board_exchange": ([_P, _P, _P, ctypes.c_double], _I),
    "dli_board_bell": ([_P], ctypes.c_uint),
    "dli_board_ring": ([_P], None),
    "dli_board_wait_bell": ([_P, ctypes.c_uint, ctypes.c_double], ctypes.c_uint),
    "dli_board_dead": ([_P], _I),
    "dli_board_close": ([_P], None),
    "dli_board_destroy": ([_P], None),
    "dli_comm_available": ([], _I),
    "dli_comm_async_error": ([_P], _I),
    "dli_comm_abort": ([_P], _I),
    "dli_comm_error_string": ([_I], ctypes.c_char_p),
    "dli_comm_unique_id": ([_P], _I),
    "dli_comm_id_bytes": ([], _I),
    "dli_comm_init": ([_P, _P, _I, _I], _I),
    "dli_comm_destroy": ([_P], _I),
    "dli_comm_exchange": ([_P, _P, _I, _P, _P, _P, _I, _P, _P, _P], _I),
    "dli_ipc_handle_bytes": ([], _I),
    "dli_ipc_create": ([_I, _I, _P, ctypes.c_char_p], _P),
    "dli_ipc_handles": ([_P, _P], _I),
    "dli_ipc_connect": ([_P, _P], _I),
    "dli_ipc_exchange": ([_P, _P, _I, _P, _P, _P, _I, _P, _P, _P], _I),
    "dli_ipc_pending": ([_P, _I], _LL),
    "dli_ipc_abort": ([_P, ctypes.c_double], _I),
    "dli_ipc_stats": ([_P, _P], None),
    "dli_ipc_error": ([_P], _I),
    "dli_ipc_ep": ([_P, _P, _I, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _I], _I),
    "dli_ipc_set_wait": ([_P, ctypes.c_double], None),
    "dli_ipc_debug_bump_seq": ([_P, _P, _I, _LL], _I),
    "dli_ipc_mem_kind": ([_P], _I),
    "dli_ipc_ep_bytes": ([_I, _I], _LL),
    "dli_ipc_host_flags": ([_P], _I),
    "dli_ipc_destroy": ([_P], None),
}


def lib():
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            from ..ops._native import ensure_current
            ensure_current(LIB_PATH, "runtime")
            L = ctypes.CDLL(str(LIB_PATH))
            for name, (args, res) in _SIGS.items():
                fn = getattr(L, name)
                fn.argtypes = args
                fn.restype = res
            _lib = L
    return _lib


def _np_ptr(a: np.ndarray) -> int:
    return a.ctypes.data              # plain int: ctypes converts it for c_void_p arguments


class BlockManager:
    """Paged KV allocator (C++). Sequence ids are arbitrary 64-bit ints."""

    def __init__(self, num_blocks: int, block_size: int):
        self._h = lib().dli_bm_create(int(num_blocks), int(block_size))
        if not self._h:
            raise ValueError("invalid block manager geometry")
        self.num_blocks = int(num_blocks)
        self.block_size = int(block_size)

    def __del__(self):
        h, self._h = getattr(self, "_h", None), None
        if h and _lib is not None:
            _lib.dli_bm_destroy(h)

    @property
    def num_free(self) -> int:
        return lib().dli_bm_num_free(self._h)

    def blocks_needed(self, seq_id: int, total_tokens: int) -> int:
        return lib().dli_bm_blocks_needed(self._h, seq_id, total_tokens)

    def ensure(self, seq_id: int, total_tokens: int) -> bool:
        return lib().dli_bm_ensure(self._h, seq_id, total_tokens) >= 0

    def ensure_batch(self, seq_ids: np.ndarray, totals: np.ndarray) -> int:
        """``ensure`` for each (seq, total) in order, stopping at the first that does not
        fit; returns how many succeeded."""
        ids = np.ascontiguousarray(seq_ids, dtype=np.int64)
        t = np.ascontiguousarray(totals, dtype=np.int32)
        return lib().dli_bm_ensure_batch(self._h, _np_ptr(ids), _np_ptr(t), ids.shape[0])

    def free(self, seq_id: int) -> int:
        return lib().dli_bm_free(self._h, seq_id)

    def free_batch(self, seq_ids: np.ndarray) -> int:
        ids = np.ascontiguousarray(seq_ids, dtype=np.int64)
        return lib().dli_bm_free_batch(self._h, _np_ptr(ids), ids.shape[0])

    def table(self, seq_id: int) -> List[int]:
        cap = max(1, self.num_blocks)
        buf = np.zeros(min(cap, 1 << 16), dtype=np.int32)
        n = lib().dli_bm_table(self._h, seq_id, _np_ptr(buf), buf.shape[0])
        return buf[:n].tolist()

    def fill_tables(self, seq_ids: Sequence[int], max_blocks: int) -> np.ndarray:
        ids = np.asarray(seq_ids, dtype=np.int64)
        out = np.zeros((len(ids), max(1, max_blocks)), dtype=np.int32)
        r = lib().dli_bm_fill_tables(self._h, _np_ptr(ids), len(ids), _np_ptr(out), out.shape[1])
        if r < 0:
            raise RuntimeError("block table wider than max_blocks")
        return out

    def decode_prepare(self, seq_ids: np.ndarray, ctx: np.ndarray, max_blocks: int):
        """One decode step's KV metadata (grow tables, new-token slots, padded tables) in
        one call. Returns (slots [n], tables [n, max_blocks], widest table), or
        (-1, i, None) when sequence i could not get a block."""
        ids = np.ascontiguousarray(seq_ids, dtype=np.int64)
        c = np.ascontiguousarray(ctx, dtype=np.int32)
        n = ids.shape[0]
        slots = np.empty(n, dtype=np.int32)
        tables = np.empty((n, max(1, max_blocks)), dtype=np.int32)
        r = lib().dli_bm_decode_prepare(self._h, _np_ptr(ids), _np_ptr(c), n, _np_ptr(slots),
                                        _np_ptr(tables), tables.shape[1])
        if r == -(n + 1):
            raise RuntimeError("block table wider than max_blocks")
        if r < 0:
            return -1, -r - 1, None
        return slots, tables, r

    # ---- automatic prefix caching (csrc/runtime/block_manager.cpp)
    def match_prefix(self, seq_id: int, hashes: np.ndarray) -> int:
        """Map the longest run of cached blocks with chain hashes ``hashes`` (uint64) as the
        first blocks of new sequence ``seq_id``; returns the number of blocks mapped."""
        h = np.ascontiguousarray(hashes, dtype=np.uint64)
        if h.shape[0] == 0:
            return 0
        return lib().dli_bm_match_prefix(self._h, int(seq_id), _np_ptr(h), h.shape[0])

    def register_prefix(self, seq_id: int, hashes: np.ndarray, first_block: int = 0) -> int:
        """Publish blocks [first_block, first_block + len(hashes)) of ``seq_id``."""
        h = np.ascontiguousarray(hashes, dtype=np.uint64)
        if h.shape[0] == 0:
            return 0
        return lib().dli_bm_register_prefix(self._h, int(seq_id), _np_ptr(h), int(first_block),
                                            h.shape[0])

    @property
    def prefix_hits(self) -> int:
        return int(lib().dli_bm_prefix_hits(self._h))

    @property
    def num_cached(self) -> int:
        return int(lib().dli_bm_num_cached(self._h))

    def slot_mapping(self, seq_ids, starts, counts) -> np.ndarray:
        ids = np.asarray(seq_ids, dtype=np.int64)
        st = np.asarray(starts, dtype=np.int32)
        ct = np.asarray(counts, dtype=np.int32)
        out = np.zeros(int(ct.sum()), dtype=np.int32)
        r = lib().dli_bm_slot_mapping(self._h, _np_ptr(ids), _np_ptr(st), _np_ptr(ct), len(ids),
                                      _np_ptr(out))
        if r < 0:
            raise RuntimeError("slot mapping beyond allocated blocks")
        return out


class DecodeCore:
    """C++ mirror of one microbatch's running sequences (``csrc/runtime/decode_core.cpp``).
    ``schedule`` returns the packed decode-step payload (StepMeta wire format) and its table
    width, ``update`` applies one token per row and returns (finished rows, EOS flags)."""

    def __init__(self, sid, ctx, out_cnt, budget, last, temp, topk, topp, seed, eos_ok,
                 eos: Optional[int], max_model_len: int, hist_cap: int):
        a = [np.ascontiguousarray(sid, np.int64), np.ascontiguousarray(ctx, np.int32),
             np.ascontiguousarray(out_cnt, np.int32), np.ascontiguousarray(budget, np.int32),
             np.ascontiguousarray(last, np.int32), np.ascontiguousarray(temp, np.float32),
             np.ascontiguousarray(topk, np.int32), np.ascontiguousarray(topp, np.float32),
             np.ascontiguousarray(seed, np.int64), np.ascontiguousarray(eos_ok, np.uint8)]
        n = a[0].shape[0]
        self._h = lib().dli_mb_create(n, *[_np_ptr(x) for x in a],
                                      -1 if eos is None else int(eos), int(max_model_len),
                                      int(hist_cap))
        if not self._h:
            raise ValueError("invalid microbatch")
        self._cols = ctypes.c_int()
        self._done = np.empty(max(1, n), np.int32)
        self._stop = np.empty(max(1, n), np.int32)

    def __del__(self):
        h, self._h = getattr(self, "_h", None), None
        if h and _lib is not None:
            _lib.dli_mb_destroy(h)

    @property
    def rows(self) -> int:
        return lib().dli_mb_rows(self._h)

    @property
    def steps(self) -> int:
        return lib().dli_mb_steps(self._h)

    def schedule(self, bm: "BlockManager", table_width: int):
        """(payload int32, table columns) or (None, failing row) when a row could not get a
        KV block."""
        L = lib()
        words = L.dli_mb_payload_words(self._h, table_width)
        out = np.empty(max(1, words), np.int32)
        r = L.dli_mb_schedule(self._h, bm._h, int(table_width), _np_ptr(out), out.shape[0],
                              ctypes.byref(self._cols))
        n = self.rows
        if r == -(n + 1):
            raise RuntimeError("decode metadata: block table wider than the table width")
        if r < 0:
            return None, int(-r - 1)
        return out[:r], self._cols.value

    def update(self, tokens: np.ndarray):
        t = np.ascontiguousarray(tokens, np.int32)
        nd = lib().dli_mb_update(self._h, _np_ptr(t), t.shape[0], _np_ptr(self._done),
                                 _np_ptr(self._stop))
        if nd < 0:
            raise ValueError(f"{t.shape[0]} tokens for a microbatch of {self.rows}")
        return self._done[:nd], self._stop[:nd]

    def row_history(self, row: int) -> List[int]:
        out = np.empty(max(1, self.steps), np.int32)
        k = lib().dli_mb_row_history(self._h, int(row), _np_ptr(out))
        return out[:k].tolist()

    def history(self) -> np.ndarray:
        n, k = self.rows, self.steps
        out = np.empty((n, k), np.int32)
        if n and k:
            lib().dli_mb_history(self._h, _np_ptr(out))
        return out

    def compact(self, drop: np.ndarray) -> int:
        d = np.ascontiguousarray(drop, np.int32)
        return lib().dli_mb_compact(self._h, _np_ptr(d), d.shape[0])


_DT = {"BF16": torch.bfloat16, "F16": torch.float16, "F32": torch.float32, "I32": torch.int32,
       "I64": torch.int64, "U8": torch.uint8, "I8": torch.int8}


class SafetensorsFile:
    def __init__(self, path: str):
        self.path = str(path)
        self._h = lib().dli_st_open(self.path.encode())
        if not self._h:
            raise IOError(f"cannot open safetensors file {path}")
        self.meta: Dict[str, tuple] = {}
        self._index: Dict[str, int] = {}
        name = ctypes.create_string_buffer(512)
        dt = ctypes.create_string_buffer(16)
        shape = (ctypes.c_longlong * 8)()
        nd, nb = ctypes.c_int(), ctypes.c_longlong()
        for i in range(lib().dli_st_count(self._h)):
            lib().dli_st_info(self._h, i, name, 512, dt, 16, ctypes.byref(shape), ctypes.byref(nd),
                              ctypes.byref(nb))
            n = name.value.decode()
            self.meta[n] = (dt.value.decode(), tuple(shape[d] for d in range(nd.value)), nb.value)
            self._index[n] = i

    def close(self):
        if self._h:
            lib().dli_st_close(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass

    def keys(self):
        return list(self.meta)

    def load(self, names=None, device="cpu") -> Dict[str, torch.Tensor]:
        names = list(self.meta) if names is None else list(names)
        dev = torch.device(device)
        out = {n: torch.empty(self.meta[n][1], dtype=_DT[self.meta[n][0]], device=dev)
               for n in names}
        if dev.type == "cuda":
            idx = (ctypes.c_int * len(names))(*[self._index[n] for n in names])
            ptrs = (ctypes.c_void_p * len(names))(*[out[n].data_ptr() for n in names])
            stream = torch.cuda.current_stream(dev).cuda_stream
            r = lib().dli_st_load_to_device(self._h, idx, ptrs, len(names), stream)
            if r < 0:
                raise RuntimeError(f"device load failed ({r})")
        else:
            for n in names:
                if lib().dli_st_copy_to_host(self._h, self._index[n],
                                             ctypes.c_void_p(out[n].data_ptr())) != 0:
                    raise RuntimeError(f"host load failed for {n}")
        return out

    def load_rows(self, name: str, lo: int, hi: int, device="cpu") -> torch.Tensor:
        """Rows [lo, hi) of a row-major tensor (e.g. one rank's vocabulary slice of the LM
        head) without reading the rest of it: a contiguous byte range of the file."""
        dt, shape, nbytes = self.meta[name]
        if not shape or not (0 <= lo <= hi <= shape[0]):
            raise ValueError(f"rows [{lo}, {hi}) outside {name} {shape}")
        row = nbytes // shape[0]
        dev = torch.device(device)
        out = torch.empty((hi - lo, *shape[1:]), dtype=_DT[dt], device=dev)
        if hi == lo:
            return out
        stream = torch.cuda.current_stream(dev).cuda_stream if dev.type == "cuda" else None
        r = lib().dli_st_load_range(self._h, self._index[name], lo * row, (hi - lo) * row,
                                    ctypes.c_void_p(out.data_ptr()), stream,
                                    1 if dev.type == "cuda" else 0)
        if r < 0:
            raise RuntimeError(f"row load failed for {name} ({r})")
        return out


class ShmRing:
    """Broadcast ring in POSIX shared memory (``csrc/runtime/shm_ring.cpp``): one producer
    publishes byte messages, every consumer reads each of them in order. ``create`` on the
    producer, ``open(index)`` on consumer ``index``; waits back off to sleeps and fail
    (``TimeoutError``) when the peer process is gone or ``timeout_s`` passes."""

    def __init__(self, handle, name: str, producer: bool):
        self._h, self.name, self.producer = handle, name, producer
        self.slot_bytes = int(lib().dli_ring_slot_bytes(handle))
        self._buf = np.empty(self.slot_bytes, dtype=np.uint8)

    @classmethod
    def create(cls, name: str, slots: int, slot_bytes: int, consumers: int) -> "ShmRing":
        h = lib().dli_ring_create(name.encode(), int(slots), int(slot_bytes), int(consumers))
        if not h:
            raise OSError(f"cannot create shared-memory ring {name}")
        return cls(h, name, True)

    @classmethod
    def open(cls, name: str, index: int, timeout_s: float = 120.0) -> "ShmRing":
        import time
        t0 = time.monotonic()
        while True:
            h = lib().dli_ring_open(name.encode(), int(index))
            if h:
                return cls(h, name, False)
            if time.monotonic() - t0 > timeout_s:
                raise OSError(f"cannot open shared-memory ring {name}")
            time.sleep(0.01)

    def unlink(self):
        lib().dli_ring_unlink(self._h)

    def publish(self, data: np.ndarray, timeout_s: float = 600.0) -> None:
        a = np.ascontiguousarray(data)
        r = lib().dli_ring_publish(self._h, _np_ptr(a), a.nbytes, float(timeout_s))
        if r == -1:
            raise ValueError(f"message of {a.nbytes} B exceeds ring slot {self.slot_bytes} B")
        if r == -2:
            raise TimeoutError("control ring: a consumer stopped reading (dead or hung)")
        if r == -3:
            raise EOFError("control ring closed")

    def consume(self, timeout_s: float = 0.0) -> np.ndarray:
        """Next message as a uint8 view of an internal buffer (valid until the next call).
        ``timeout_s`` = 0 waits as long as the producer process is alive."""
        n = lib().dli_ring_consume(self._h, _np_ptr(self._buf), self._buf.nbytes,
                                   float(timeout_s))
        if n == -2:
            raise TimeoutError("control ring: producer gone or timeout")
        if n == -3:
            raise EOFError("control ring closed")
        if n < 0:
            raise RuntimeError(f"control ring consume failed ({n})")
        return self._buf[:n]

    @property
    def published(self) -> int:
        return int(lib().dli_ring_published(self._h))

    @property
    def min_consumed(self) -> int:
        return int(lib().dli_ring_min_consumed(self._h))

    def dead(self) -> int:
        """-1 while every process on the ring lives; else the index of a consumer whose
        process is gone, or 1000 for the producer."""
        return int(lib().dli_ring_dead(self._h)) if self._h else -1

    def close(self):
        if self._h:
            lib().dli_ring_close(self._h)

    def destroy(self):
        h, self._h = self._h, None
        if h and _lib is not None:
            _lib.dli_ring_destroy(h)

    def __del__(self):
        try:
            self.destroy()
        except Exception:  # noqa: BLE001
            pass


class LockstepBoard:
    """Per-step all-gather of a few int64 words between the processes of one node, in POSIX
    shared memory (``csrc/runtime/lockstep.cpp``), plus a doorbell idle ranks sleep on. The
    expert-parallel ranks' lockstep control plane: ``create`` on rank 0, ``open`` on the
    others (after the name was shared), ``join(rank)`` on every rank, ``unlink`` once all
    joined. Waits fail with ``TimeoutError`` / ``PeerGone`` instead of hanging."""

    VALS = 4

    class PeerGone(RuntimeError):
        pass

    def __init__(self, handle, name: str):
        self._h, self.name = handle, name
        self.world = int(lib().dli_board_world(handle))
        self._out = np.zeros(self.world * self.VALS, dtype=np.int64)
        self._in = np.zeros(self.VALS, dtype=np.int64)

    @classmethod
    def create(cls, name: str, world: int) -> "LockstepBoard":
        h = lib().dli_board_create(name.encode(), int(world))
        if not h:
            raise OSError(f"cannot create lockstep board {name}")
        return cls(h, name)

    @classmethod
    def open(cls, name: str, timeout_s: float = 60.0) -> "LockstepBoard":
        import time
        t0 = time.monotonic()
        while True:
            h = lib().dli_board_open(name.encode())
            if h:
                return cls(h, name)
            if time.monotonic() - t0 > timeout_s:
                raise OSError(f"cannot open lockstep board {name}")
            time.sleep(0.01)

    def join(self, rank: int) -> None:
        if lib().dli_board_join(self._h, int(rank)) != 0:
            raise ValueError(f"rank {rank} outside the board's {self.world} ranks")

    def unlink(self) -> None:
        lib().dli_board_unlink(self._h)

    def exchange(self, words: Sequence[int], timeout_s: float = 120.0) -> np.ndarray:
        """Publish ``words`` (<= 4 ints), return every rank's words [world, 4] (a view of a
        buffer the next exchange overwrites)."""
        self._in[:] = 0
        self._in[:len(words)] = words
        r = lib().dli_board_exchange(self._h, _np_ptr(self._in), _np_ptr(self._out),
                                     float(timeout_s))
        if r == -2:
            raise self.PeerGone(f"lockstep peer rank {self.dead()} exited")
        if r == -1:
            raise TimeoutError(f"lockstep exchange timed out after {timeout_s} s")
        if r != 0:
            raise RuntimeError(f"lockstep board closed or not joined ({r})")
        return self._out.reshape(self.world, self.VALS)

    def bell(self) -> int:
        return int(lib().dli_board_bell(self._h))

    def ring(self) -> None:
        lib().dli_board_ring(self._h)

    def wait_bell(self, seen: int, timeout_s: float) -> int:
        """Sleep (futex) until the doorbell moves past ``seen`` or ``timeout_s`` passes."""
        return int(lib().dli_board_wait_bell(self._h, int(seen) & 0xffffffff,
                                             float(timeout_s)))

    def dead(self) -> int:
        return int(lib().dli_board_dead(self._h)) if self._h else -1

    def close(self) -> None:
        if self._h:
            lib().dli_board_close(self._h)

    def destroy(self) -> None:
        h, self._h = self._h, None
        if h and _lib is not None:
            _lib.dli_board_destroy(h)

    def __del__(self):
        try:
            self.destroy()
        except Exception:  # noqa: BLE001
            pass


class RcclComm:
    """A pipeline's RCCL communicator driven directly (``csrc/runtime/comm.cpp``): a tick's
    sends and receives go out in one ncclGroupStart/End on the caller's stream (the stage's
    compute stream), ordered with the kernels around them without events or host waits.
    ``uid`` is the 128-byte id from ``RcclComm.unique_id()`` on rank 0, shared by every rank
    (the pipeline ships it over its gloo control group)."""

    def __init__(self, uid: bytes, world: int, rank: int):
        L = lib()
        if not L.dli_comm_available():
            raise RuntimeError("RCCL (librccl.so.1) could not be loaded")
        h = ctypes.c_void_p()
        buf = ctypes.create_string_buffer(bytes(uid), len(uid))
        r = L.dli_comm_init(ctypes.byref(h), buf, int(world), int(rank))
        if r != 0:
            raise RuntimeError(f"ncclCommInitRank failed: {L.dli_comm_error_string(r).decode()}")
        self._h = h.value
        self.world, self.rank = world, rank
        # the tick thread enqueues exchanges while the pipeline watchdog may abort the
        # communicator: every use of the handle holds this lock, and an aborted handle is
        # never dereferenced again (exchange raises instead)
        self._lock = threading.Lock()

    @staticmethod
    def available() -> bool:
        return bool(lib().dli_comm_available())

    @staticmethod
    def unique_id() -> bytes:
        L = lib()
        n = L.dli_comm_id_bytes()
        buf = ctypes.create_string_buffer(n)
        r = L.dli_comm_unique_id(buf)
        if r != 0:
            raise RuntimeError(f"ncclGetUniqueId failed: {L.dli_comm_error_string(r).decode()}")
        return buf.raw

    def exchange(self, sends, recvs, stream: int) -> None:
        """``sends`` / ``recvs`` = [(device tensor, peer)]; enqueued on ``stream`` (an int
        hipStream_t, e.g. ``torch.cuda.current_stream().cuda_stream``)."""
        def pack(items):
            n = len(items)
            ptrs = (ctypes.c_void_p * max(n, 1))(*[t.data_ptr() for t, _ in items])
            nbytes = (ctypes.c_longlong * max(n, 1))(*[t.numel() * t.element_size()
                                                      for t, _ in items])
            peers = (ctypes.c_int * max(n, 1))(*[int(p) for _, p in items])
            return n, ptrs, nbytes, peers
        ns, sp, sb, spe = pack(sends)
        nr, rp, rb, rpe = pack(recvs)
        with self._lock:
            if self._h is None:
                raise RuntimeError("RCCL exchange on an aborted / closed communicator")
            r = lib().dli_comm_exchange(self._h, ctypes.c_void_p(stream), ns, sp, sb, spe, nr,
                                        rp, rb, rpe)
        if r != 0:
            raise RuntimeError(f"RCCL exchange failed: {lib().dli_comm_error_string(r).decode()}")

    BUSY = 1        # async_error(): an exchange is being enqueued on another thread

    def async_error(self) -> int:
        """0 while healthy, -(ncclResult_t) of the communicator's asynchronous error, or
        ``BUSY`` while another thread holds the handle inside an exchange (the caller decides
        how long an enqueue may stay blocked: ``PipeChannel._watch`` aborts a stuck one)."""
        if not self._lock.acquire(timeout=0.05):
            return self.BUSY
        try:
            return int(lib().dli_comm_async_error(self._h)) if self._h is not None else 0
        finally:
            self._lock.release()

    def abort(self, wait_s: float = 1.0) -> None:
        """ncclCommAbort: release the communicator without waiting for peers (a dead
        neighbour); queued RCCL kernels return so the stream drains. An exchange being
        enqueued on another thread gets ``wait_s`` to leave the handle; if it is still blocked
        there (a group end waiting on the dead peer) the handle is marked dead and aborted
        anyway — the abort is what releases that blocked call, so waiting for it would turn a
        fast failure into a hang. Later exchanges raise instead of touching the handle."""
        got = self._lock.acquire(timeout=max(0.0, float(wait_s)))
        try:
            h, self._h = self._h, None
            if h is not None:
                lib().dli_comm_abort(h)
        finally:
            if got:
                self._lock.release()

    def close(self) -> None:
        with self._lock:
            h, self._h = self._h, None
            if h is not None:
                lib().dli_comm_destroy(h)

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass


def _pack_io(items):
    n = len(items)
    ptrs = (ctypes.c_void_p * max(n, 1))(*[t.data_ptr() for t, _ in items])
    nbytes = (ctypes.c_longlong * max(n, 1))(*[t.numel() * t.element_size() for t, _ in items])
    peers = (ctypes.c_int * max(n, 1))(*[int(p) for _, p in items])
    return n, ptrs, nbytes, peers


class IpcEndpoint:
    """Device-memory mailbox transport of one rank (``csrc/runtime/ipc.cpp``): one mailbox
    per directed edge in the receiver's HBM (uncached: no L2 keeps a copy of a line a peer
    writes over xGMI), filled by a stream-ordered put kernel and handed over by READY / FREE
    binary semaphores (bounded wait kernels; no host-side sequence numbers, so captured
    exchanges replay correctly). Every message carries a device-side sequence number that
    the receiver checks: a stale or out-of-order mailbox sets ``error()`` instead of
    yielding wrong activations. FIFO per edge (RCCL's matching rule), everything enqueued on
    the caller's stream.

    Setup is three steps so the caller can move the handles over any side channel:
    ``ep = IpcEndpoint(world, rank, cap)``; gather ``ep.handles()`` from every rank;
    ``ep.connect(all_handles)``. ``cap[src][dst]`` = mailbox bytes of edge src -> dst
    (0 = no edge), the same matrix on every rank. ``host_prefix``: keep the flag words in
    POSIX shared-memory pages (host-visible progress; ``abort()`` releases a dead peer's
    waits)."""

    ERR_WAIT, ERR_SEQ, ERR_ABORT = 1, 2, 4
    MEM_KINDS = {0: "coarse", 1: "fine", 2: "uncached"}

    def __init__(self, world: int, rank: int, cap, host_prefix: str = ""):
        L = lib()
        m = np.ascontiguousarray(np.asarray(cap, dtype=np.int64).reshape(world, world))
        self.cap = m
        self._h = L.dli_ipc_create(int(world), int(rank), _np_ptr(m), host_prefix.encode())
        if not self._h:
            raise RuntimeError("IPC endpoint: allocation failed")
        self.world, self.rank = world, rank
        self.host_flags = bool(L.dli_ipc_host_flags(self._h))
        self.mem_kind = self.MEM_KINDS.get(int(L.dli_ipc_mem_kind(self._h)), "?")

    def handles(self) -> bytes:
        hb = lib().dli_ipc_handle_bytes()
        buf = ctypes.create_string_buffer(2 * hb)
        r = lib().dli_ipc_handles(self._h, buf)
        if r < 0:
            raise RuntimeError(f"hipIpcGetMemHandle failed (hipError {-r})")
        return buf.raw

    def connect(self, all_handles: Sequence[bytes]) -> None:
        blob = b"".join(bytes(h) for h in all_handles)
        buf = ctypes.create_string_buffer(blob, len(blob))
        r = lib().dli_ipc_connect(self._h, buf)
        if r != 0:
            raise RuntimeError(f"IPC connect failed ({r}: hipIpcOpenMemHandle / shm map)")

    def exchange(self, sends, recvs, stream: int) -> None:
        """``sends`` / ``recvs`` = [(device tensor, peer)], enqueued on ``stream``."""
        ns, sp, sb, spe = _pack_io(sends)
        nr, rp, rb, rpe = _pack_io(recvs)
        r = lib().dli_ipc_exchange(self._h, ctypes.c_void_p(stream), ns, sp, sb, spe, nr, rp,
                                   rb, rpe)
        if r != 0:
            raise RuntimeError(f"IPC exchange failed ({r})" + (
                ": message larger than the edge's slot" if r == -1003 else ""))

    def pending(self, peer: int) -> int:
        """Host-flag mode: 1 while a message from ``peer`` waits in this rank's mailbox."""
        return int(lib().dli_ipc_pending(self._h, int(peer)))

    def abort(self, timeout_s: float = 5.0) -> None:
        """Set every flag this rank's queue could be waiting on (a dead peer's mailboxes):
        the blocked exchange completes (with stale payload) so the stream drains."""
        r = lib().dli_ipc_abort(self._h, float(timeout_s))
        if r != 0:
            raise RuntimeError(f"IPC abort failed ({r})")

    @staticmethod
    def ep_bytes(cap_rows: int, row_bytes: int) -> int:
        return int(lib().dli_ipc_ep_bytes(int(cap_rows), int(row_bytes)))

    def ep(self, stream: int, ret: bool, row_bytes: int, send_x, send_e, send_base, send_cnt,
           recv_x, recv_e, recv_base, recv_cap, recv_cnt, cap_rows, in_cap_rows,
           send_cap: Optional[int] = None) -> None:
        """Expert-parallel dispatch (``ret`` False) or return over the mailboxes (see
        ``dli_ipc_ep``): row counts stay on the device (``send_cnt`` / ``recv_cnt`` int32
        tensors), only the routed rows move. ``send_cap``: rows of each per-peer send region
        (a returned count is clamped to it)."""
        W = self.world
        ia = lambda v: (ctypes.c_int * W)(*[int(x) for x in v])  # noqa: E731
        if send_cap is None:
            send_cap = max(int(c) for c in cap_rows)
        r = lib().dli_ipc_ep(self._h, ctypes.c_void_p(stream), int(bool(ret)), int(row_bytes),
                             send_x.data_ptr(), send_e.data_ptr() if send_e is not None else None,
                             ia(send_base), send_cnt.data_ptr(), recv_x.data_ptr(),
                             recv_e.data_ptr() if recv_e is not None else None, ia(recv_base),
                             ia(recv_cap), recv_cnt.data_ptr(), ia(cap_rows), ia(in_cap_rows),
                             int(send_cap))
        if r != 0:
            raise RuntimeError(f"IPC expert exchange failed ({r})")

    def error(self) -> int:
        """Error bits raised by this rank's queue so far (0 = healthy): ``ERR_WAIT`` a bounded
        wait ran out of budget (a peer stopped), ``ERR_SEQ`` a message's sequence number or
        size did not match (stale / lost / mis-ordered), ``ERR_ABORT`` the ring was aborted.
        One load of a pinned host word: cheap enough for every tick."""
        return int(lib().dli_ipc_error(self._h))

    def set_wait(self, seconds: float) -> None:
        """Budget of the wait kernels enqueued from now on."""
        lib().dli_ipc_set_wait(self._h, float(seconds))

    def debug_bump_seq(self, peer: int, stream: int, d: int = 1) -> None:
        """Test hook: the next message to ``peer`` carries a wrong sequence number."""
        r = lib().dli_ipc_debug_bump_seq(self._h, ctypes.c_void_p(stream), int(peer), int(d))
        if r != 0:
            raise RuntimeError(f"IPC bump failed ({r})")

    def stats(self) -> Dict[str, int]:
        out = (ctypes.c_longlong * 3)()
        lib().dli_ipc_stats(self._h, out)
        return {"sends": out[0], "recvs": out[1], "bytes_out": out[2]}

    def close(self) -> None:
        h, self._h = getattr(self, "_h", None), None
        if h and _lib is not None:
            _lib.dli_ipc_destroy(h)

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass
