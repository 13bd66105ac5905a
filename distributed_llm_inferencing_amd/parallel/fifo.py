"""Tag-blind FIFO data plane on the host: the CPU model of the device mailbox transport.

``ShmMailboxTransport`` runs the exact protocol of ``csrc/runtime/ipc.cpp`` — one mailbox per
directed edge, a READY / FREE binary-semaphore pair, sends then receives in issue order —
with the host as the "queue": a wait blocks the caller the way a ``hipStreamWaitValue64``
blocks the stream. Since a HIP stream also executes its waits in issue order, a schedule that
completes here completes on the GPU queues, and one that deadlocks here deadlocks there.

Matching is strictly FIFO per (src, dst) and ignores tags, which is RCCL's rule as well:
gloo matches point-to-point messages by (peer, tag), so a pair of ranks whose send and
receive orders diverge passes every gloo test and corrupts (or hangs) on RCCL. Here every
message carries its byte count, and a receive whose buffer size differs from the message at
the head of its edge raises ``FifoMismatch`` naming both sides — the order bug surfaces on
CPU, in a test (``tests/test_fifo_transport.py``).

Mailboxes live in POSIX shared memory (``multiprocessing.shared_memory``): rank r's segment
holds its inbound mailboxes and its flag words; peers attach after a barrier.
"""
from __future__ import annotations

import time
from multiprocessing import shared_memory
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

_LINE = 8                  # int64 words per flag (one 64-byte line each)


class FifoMismatch(RuntimeError):
    pass


def _segment(name: str, size: int = 0) -> shared_memory.SharedMemory:
    """Create (size > 0) or attach a segment WITHOUT the resource tracker: Python 3.10
    registers created and attached segments alike with a tracker the spawned ranks may
    share, which then double-unregisters (or unlinks) them; here the creating rank owns the
    segment and unlinks it in ``close()``."""
    from multiprocessing import resource_tracker
    reg = resource_tracker.register
    resource_tracker.register = lambda *a, **k: None
    try:
        if size:
            return shared_memory.SharedMemory(name=name, create=True, size=size)
        return shared_memory.SharedMemory(name=name)
    finally:
        resource_tracker.register = reg


class ShmMailboxTransport:
    """One rank's endpoint. ``cap[src][dst]`` = mailbox bytes of edge src -> dst (0 = none),
    the same matrix on every rank. Create on every rank, barrier, then ``connect()``."""

    def __init__(self, world: int, rank: int, cap, prefix: str, timeout_s: float = 120.0):
        self.world, self.rank = world, rank
        self.cap = np.asarray(cap, dtype=np.int64).reshape(world, world)
        self.prefix = prefix
        self.timeout_s = timeout_s
        W = world
        # layout: flags [READY[src] x W][FREE[dst] x W] (one line each), then per inbound
        # edge a 16-byte header {size, sequence} + the mailbox (ipc.cpp's message header)
        self._flag_bytes = 2 * W * _LINE * 8
        self._off = {}
        off = self._flag_bytes
        for s in range(W):
            c = int(self.cap[s, rank])
            if c > 0:
                self._off[s] = off
                off += 16 + ((c + 7) // 8) * 8
        self._size = off
        self.shm = _segment(self._name(rank), off)
        flags = np.ndarray((2 * W * _LINE,), dtype=np.int64, buffer=self.shm.buf)
        flags[:] = 0
        for d in range(W):
            flags[(W + d) * _LINE] = 1            # every outbound mailbox starts free
        self.peers: Dict[int, shared_memory.SharedMemory] = {}
        self.sends = self.recvs = 0
        self.bytes_out = 0
        self.seq_out = [0] * W          # per-edge sequence numbers, as ipc.cpp keeps on device
        self.seq_in = [0] * W
        self.err = 0
        self.mem_kind = "shm"

    def _name(self, r: int) -> str:
        return f"{self.prefix.strip('/')}_{r}"

    def connect(self) -> None:
        for p in range(self.world):
            if p == self.rank:
                continue
            if self.cap[self.rank, p] > 0 or self.cap[p, self.rank] > 0:
                self.peers[p] = _segment(self._name(p))

    # ---- flag words ------------------------------------------------------------------
    def _flags(self, shm) -> np.ndarray:
        return np.ndarray((2 * self.world * _LINE,), dtype=np.int64, buffer=shm.buf)

    def _wait(self, arr: np.ndarray, idx: int, what: str) -> None:
        t0 = time.monotonic()
        spins = 0
        while arr[idx] != 1:
            if self.err & 4:             # aborted: sticky, every later wait passes (as on device)
                return
            spins += 1
            if spins > 200:
                time.sleep(0.0002 if spins < 5000 else 0.002)
            if time.monotonic() - t0 > self.timeout_s:
                raise TimeoutError(f"rank {self.rank}: {what} not signalled within "
                                   f"{self.timeout_s} s (peer dead or schedule deadlocked)")
        arr[idx] = 0

    # ---- data plane ------------------------------------------------------------------
    def _peer_off(self, peer: int) -> int:
        """Offset of MY mailbox inside ``peer``'s segment (edge me -> peer)."""
        W = self.world
        off = self._flag_bytes
        for s in range(W):
            c = int(self.cap[s, peer])
            if s == self.rank:
                return off
            if c > 0:
                off += 16 + ((c + 7) // 8) * 8
        raise KeyError(peer)

    def send(self, t: torch.Tensor, peer: int) -> None:
        W = self.world
        b = t.detach().contiguous().view(-1).view(torch.uint8).numpy() if t.numel() else \
            np.zeros(0, np.uint8)
        if b.nbytes > self.cap[self.rank, peer]:
            raise ValueError(f"rank {self.rank} -> {peer}: message of {b.nbytes} B exceeds the "
                             f"mailbox ({self.cap[self.rank, peer]} B)")
        mine = self._flags(self.shm)
        self._wait(mine, (W + peer) * _LINE, f"FREE[{self.rank}->{peer}]")
        pshm = self.peers[peer]
        off = self._peer_off(peer)
        self.seq_out[peer] += 1
        np.ndarray((2,), np.int64, buffer=pshm.buf, offset=off)[:] = (b.nbytes, self.seq_out[peer])
        if b.nbytes:
            np.ndarray((b.nbytes,), np.uint8, buffer=pshm.buf, offset=off + 16)[:] = b
        self._flags(pshm)[self.rank * _LINE] = 1        # READY in the peer's page
        self.sends += 1
        self.bytes_out += b.nbytes

    def recv(self, buf: torch.Tensor, peer: int) -> None:
        mine = self._flags(self.shm)
        self._wait(mine, peer * _LINE, f"READY[{peer}->{self.rank}]")
        off = self._off[peer]
        n, seq = (int(v) for v in np.ndarray((2,), np.int64, buffer=self.shm.buf, offset=off))
        self._check_seq(peer, seq)
        want = buf.numel() * buf.element_size()
        if n != want:
            raise FifoMismatch(f"rank {self.rank} <- {peer}: the message at the head of the edge "
                               f"has {n} B, the receive posted {want} B (send / receive order "
                               f"differs between the two ranks)")
        if n:
            src = np.ndarray((n,), np.uint8, buffer=self.shm.buf, offset=off + 16)
            buf.view(-1).view(torch.uint8).copy_(torch.from_numpy(src.copy()))
        self._flags(self.peers[peer])[(self.world + self.rank) * _LINE] = 1   # FREE
        self.recvs += 1

    def _check_seq(self, peer: int, seq: int) -> None:
        self.seq_in[peer] += 1
        if seq != self.seq_in[peer]:
            self.err |= 2
            raise FifoMismatch(f"rank {self.rank} <- {peer}: message sequence {seq}, expected "
                               f"{self.seq_in[peer]} (stale, lost or duplicated message)")

    # ---- the device endpoint's error / test surface (ipc.cpp) --------------------------
    def error(self) -> int:
        return self.err

    def set_wait(self, seconds: float) -> None:
        self.timeout_s = float(seconds)

    def debug_bump_seq(self, peer: int, stream=None, d: int = 1) -> None:
        self.seq_out[peer] += int(d)

    def abort(self, timeout_s: float = 5.0) -> None:
        """Release every wait of this rank (a dead peer): set all of its flags."""
        self.err |= 4
        flags = self._flags(self.shm)
        for i in range(2 * self.world):
            flags[i * _LINE] = 1

    # ---- variable-length messages (expert-parallel rows: the count travels with them) ---
    def send_raw(self, b: np.ndarray, peer: int) -> None:
        b = np.ascontiguousarray(b).reshape(-1).view(np.uint8)
        self.send(torch.from_numpy(b) if b.nbytes else torch.zeros(0, dtype=torch.uint8), peer)

    def recv_raw(self, peer: int) -> np.ndarray:
        """The message at the head of edge peer -> me, whatever its size."""
        mine = self._flags(self.shm)
        self._wait(mine, peer * _LINE, f"READY[{peer}->{self.rank}]")
        off = self._off[peer]
        n, seq = (int(v) for v in np.ndarray((2,), np.int64, buffer=self.shm.buf, offset=off))
        self._check_seq(peer, seq)
        out = np.ndarray((n,), np.uint8, buffer=self.shm.buf, offset=off + 16).copy()
        self._flags(self.peers[peer])[(self.world + self.rank) * _LINE] = 1   # FREE
        self.recvs += 1
        return out

    def ep(self, stream, ret: bool, row_bytes: int, send_x, send_e, send_base, send_cnt,
           recv_x, recv_e, recv_base, recv_cap, recv_cnt, cap_rows, in_cap_rows,
           send_cap=None) -> None:
        """Host model of ``IpcEndpoint.ep`` (csrc/runtime/ipc.cpp ``dli_ipc_ep``): the same
        message order and per-edge FIFO, counts read from the tensors."""
        W, me = self.world, self.rank
        sx = send_x.view(torch.uint8).view(-1, row_bytes)
        rx = recv_x.view(torch.uint8).view(-1, row_bytes)

        def msg(rows: torch.Tensor, ids: Optional[torch.Tensor]) -> np.ndarray:
            n = np.array([rows.shape[0]], np.int64).view(np.uint8)
            parts = [n]
            if ids is not None:
                parts.append(ids.contiguous().numpy().view(np.uint8))
            parts.append(rows.contiguous().numpy().reshape(-1))
            return np.concatenate(parts)

        def unpack(b: np.ndarray, with_ids: bool):
            n = int(b[:8].view(np.int64)[0])
            o = 8
            ids = None
            if with_ids:
                ids = torch.from_numpy(b[o:o + 4 * n].view(np.int32).copy())
                o += 4 * n
            rows = torch.from_numpy(b[o:o + n * row_bytes].copy()).view(n, row_bytes)
            return n, ids, rows
        if not ret:
            for p in range(W):
                if p == me:
                    continue
                c = int(send_cnt[p])
                if c > cap_rows[p]:
                    raise ValueError(f"expert bucket {me}->{p}: {c} rows > capacity {cap_rows[p]}")
                b0 = int(send_base[p])
                self.send_raw(msg(sx[b0:b0 + c], send_e[b0:b0 + c]), p)
            c = int(send_cnt[me])
            rb, sb = int(recv_base[me]), int(send_base[me])
            rx[rb:rb + c] = sx[sb:sb + c]
            recv_e[rb:rb + int(recv_cap[me])] = -1
            recv_e[rb:rb + c] = send_e[sb:sb + c]
            recv_cnt[me] = c
            for q in range(W):
                if q == me:
                    continue
                n, ids, rows = unpack(self.recv_raw(q), True)
                rb = int(recv_base[q])
                if n > int(recv_cap[q]):
                    raise ValueError(f"expert rows {q}->{me}: {n} > region {recv_cap[q]}")
                rx[rb:rb + n] = rows
                recv_e[rb:rb + int(recv_cap[q])] = -1
                recv_e[rb:rb + n] = ids
                recv_cnt[q] = n
            return
        for q in range(W):
            if q == me:
                continue
            c, rb = int(recv_cnt[q]), int(recv_base[q])
            self.send_raw(msg(rx[rb:rb + c], None), q)
        c, rb, sb = int(recv_cnt[me]), int(recv_base[me]), int(send_base[me])
        sx[sb:sb + c] = rx[rb:rb + c]
        for p in range(W):
            if p == me:
                continue
            n, _, rows = unpack(self.recv_raw(p), False)
            sb = int(send_base[p])
            sx[sb:sb + n] = rows

    def exchange(self, sends: Sequence[Tuple[torch.Tensor, int]],
                 recvs: Sequence[Tuple[torch.Tensor, int]], stream=None) -> None:
        """Every send, then every receive, in issue order (the device queue's order)."""
        for t, p in sends:
            self.send(t, p)
        for b, p in recvs:
            self.recv(b, p)

    def stats(self) -> dict:
        return {"sends": self.sends, "recvs": self.recvs, "bytes_out": self.bytes_out}

    def close(self) -> None:
        for p in self.peers.values():
            p.close()
        self.peers = {}
        if self.shm is not None:
            name = self.shm._name
            self.shm.close()
            try:
                import _posixshmem
                _posixshmem.shm_unlink(name)
            except (FileNotFoundError, ImportError):
                pass
            self.shm = None


def mailbox_caps(world: int, big: int, small: int, big_edges: Optional[List[Tuple[int, int]]]
                 = None) -> np.ndarray:
    """Capacity matrix: ``big`` bytes on the listed edges (default r -> r + 1, the pipeline's
    activation edges), ``small`` on every other edge, 0 on the diagonal."""
    m = np.full((world, world), int(small), dtype=np.int64)
    np.fill_diagonal(m, 0)
    for s, d in (big_edges if big_edges is not None else
                 [(r, r + 1) for r in range(world - 1)]):
        m[s, d] = int(big)
    return m
