"""Inter-stage transport for the layer-sharded pipeline.

The reference has NO inter-shard data plane (its "sharded" path runs shard 0 alone,
``worker/app.py:334-336``). Here a pipeline step moves over two planes:

* control plane (host): the head's packed ``StepMeta`` for every tick goes to every other
  stage over a separate **gloo** process group (TCP loopback, CPU tensors) the moment the
  head schedules it, so a stage's host can stage the metadata upload and enqueue its graph
  replay long before the activations arrive — no stage ever waits on its GPU to learn what
  to do next;
* data plane (device): hidden states stage r -> r+1 and sampled token ids tail -> head go by
  RCCL point-to-point over xGMI (``torch.distributed`` backend "nccl" == RCCL on ROCm), one
  grouped send/recv per rank per tick, ordered on the GPU streams: the receive is a stream
  dependency of the consumer's graph replay, never a host wait. On CPU (tests) the data
  plane is gloo as well.

Every stage learns the activation shape of tick k from tick k's metadata (rows = tokens of
the step, cols = hidden size), so the data plane carries no headers at all.
"""
from __future__ import annotations

import os
from collections import deque
from datetime import timedelta
from typing import Optional, Tuple

import numpy as np
import torch
import torch.distributed as dist

from ..engine.batch import HEADER_LEN
from ..utils import faults
from ..utils.tracing import trace_range

# header word indices (int64 units) beyond StepMeta's own first 8
H_TICK = 12


class PipeChannel:
    """Control + data planes of one pipeline rank (default process group = the stages).

    Data plane: ONE grouped ``batch_isend_irecv`` per rank per tick on the default
    communicator — {send my output of tick k-1 -> next, receive my input of tick k <- prev}
    (the tail's output is the sampled ids, sent to the head). Rank r's group at tick k pairs
    with rank r+1's and rank r-1's groups of the same tick (anti-diagonal schedule), so all
    ranks exchange together and nothing can wait on a later tick: deadlock-free. One
    communicator = one RCCL stream per rank: separate per-edge communicators would add
    streams that HIP may alias onto the same hardware queue (GPU_MAX_HW_QUEUES=4), putting
    a spinning receive in front of a send."""

    def __init__(self, device: torch.device, dtype=torch.bfloat16, max_pending: int = 8):
        self.rank = dist.get_rank()
        self.world = dist.get_world_size()
        self.device = torch.device(device)
        self.dtype = dtype
        self.nccl = dist.get_backend() == "nccl"
        # collective over all ranks (called once per engine). Idle serving ranks block on
        # the control plane between sessions: no timeout that could fire while idle.
        self.ctrl_group = dist.new_group(backend="gloo", timeout=timedelta(days=365))
        self.data_device = self.device if self.nccl else torch.device("cpu")
        self._inflight = deque()
        self._ctrl_sends = deque()
        self.max_pending = max_pending
        self.side_stream = (torch.cuda.Stream(self.device)
                            if self.nccl and self.device.type == "cuda" else None)
        if self.world > 1:
            # every rank joins one grouped ring exchange up front, so whatever point-to-point
            # communicator state RCCL builds lazily is built with all ranks present (the
            # session's first exchanges involve only some ranks)
            t = torch.full((1,), float(self.rank), device=self.data_device)
            r = torch.empty(1, device=self.data_device)
            for w in dist.batch_isend_irecv([dist.P2POp(dist.isend, t, self.next),
                                             dist.P2POp(dist.irecv, r, self.prev)]):
                w.wait()
            if int(r.item()) != self.prev:
                raise RuntimeError(f"pipeline ring check failed on rank {self.rank}")

    @property
    def next(self) -> int:
        return (self.rank + 1) % self.world

    @property
    def prev(self) -> int:
        return (self.rank - 1) % self.world

    # ------------------------------------------------------------------ control plane
    def broadcast_ctrl(self, header: np.ndarray, payload: np.ndarray) -> None:
        """Head -> every other stage (asynchronous; buffers kept until delivered)."""
        if faults.active():
            faults.check("transport.exchange", tick=int(header[H_TICK]))
        h = torch.from_numpy(np.ascontiguousarray(header, dtype=np.int64).copy())
        h[4] = int(payload.shape[0])
        p = torch.from_numpy(np.ascontiguousarray(payload, dtype=np.int32).copy())
        with trace_range("pp.ctrl"):
            for r in range(1, self.world):
                self._ctrl_sends.append((dist.isend(h, r, group=self.ctrl_group), h))
                if p.numel():
                    self._ctrl_sends.append((dist.isend(p, r, group=self.ctrl_group), p))
        # never block here: stage r consumes the message of tick j only after the head has
        # posted its data exchange of tick j (and stage r-1 has run), so a blocking drain
        # BEFORE this tick's exchange can deadlock a deep ring (8 stages: ~2 x 28 messages
        # are legitimately in flight). The head drains in reap_ctrl() after its exchange.
        self._reap(blocking_above=None)

    def _reap(self, blocking_above):
        q = self._ctrl_sends
        while q and q[0][0].is_completed():
            q.popleft()[0].wait()          # completed: returns at once, releases the Work
        if blocking_above is not None:
            while len(q) > blocking_above:
                w, _ = q.popleft()
                w.wait()

    def reap_ctrl(self) -> None:
        """Head, after posting this tick's data exchange: release delivered control messages
        and bound the backlog (safe to block now: every stage can consume the messages of
        ticks <= the one just posted)."""
        self._reap(blocking_above=64 * self.world)

    def recv_ctrl(self) -> Tuple[np.ndarray, np.ndarray]:
        h = torch.empty(HEADER_LEN, dtype=torch.int64)
        dist.recv(h, 0, group=self.ctrl_group)
        n = int(h[4])
        p = torch.empty(n, dtype=torch.int32)
        if n:
            dist.recv(p, 0, group=self.ctrl_group)
        return h.numpy(), p.numpy()

    # ------------------------------------------------------------------ data plane
    def exchange_many(self, sends, recvs):
        """Post this tick's grouped exchange. ``sends`` = [(tensor, peer, tag)] (snapshotted:
        graph outputs are static buffers), ``recvs`` = [(shape, dtype, peer, tag)]. Tags
        keep several messages between one pair apart (gloo matches per (peer, tag); RCCL
        ignores them). Returns (recv buffers, record) for ``wait_all``, or None."""
        ops, keep, bufs = [], [], []
        with trace_range("pp.exchange"):
            for t, peer, tag in sends:
                if t is None or t.numel() == 0:
                    continue
                snap = t.clone() if self.nccl else t.to("cpu")
                snap = snap.contiguous()
                keep.append(snap)
                ops.append(dist.P2POp(dist.isend, snap, peer, tag=tag))
            for shape, dt, peer, tag in recvs:
                buf = torch.empty(shape, dtype=dt, device=self.data_device)
                bufs.append(buf)
                ops.append(dist.P2POp(dist.irecv, buf, peer, tag=tag))
            if not ops:
                return None
            works = dist.batch_isend_irecv(ops)
        rec = [works, keep, False]        # [works, snapshots, waited]
        self._inflight.append(rec)
        while len(self._inflight) > self.max_pending:
            self._finish(self._inflight.popleft())
        return bufs, rec

    def exchange(self, send: Optional[torch.Tensor], recv_shape: Optional[tuple],
                 recv_dtype=None):
        """Ring-only form: {send -> next, receive <- prev} (tag 1)."""
        r = self.exchange_many([(send, self.next, 1)] if send is not None else [],
                               [(recv_shape, recv_dtype or self.dtype, self.prev, 1)]
                               if recv_shape is not None else [])
        if r is None:
            return None
        bufs, rec = r
        return (bufs[0] if bufs else None), rec

    def wait_all(self, handle):
        """Receive buffers of an exchange (on RCCL a stream dependency, not a host wait)."""
        bufs, rec = handle
        self._finish(rec)
        return [b if b.device == self.device else b.to(self.device) for b in bufs]

    def _finish(self, rec) -> None:
        # a gloo Work must be waited exactly once (a second wait on a completed receive
        # blocks forever); an RCCL wait is a dependency of the CURRENT stream and idempotent,
        # so it is always issued (the caller's stream may not have waited yet)
        if self.nccl or not rec[2]:
            for w in rec[0]:
                w.wait()
            rec[2] = True

    def wait(self, handle) -> torch.Tensor:
        """Input of this tick: on RCCL a stream dependency of the replay, not a host wait."""
        buf, rec = handle
        self._finish(rec)
        return buf if buf.device == self.device else buf.to(self.device)

    def to_host(self, handle) -> np.ndarray:
        """Head: the tail's sampled ids on the host, synchronised on a side stream so the
        compute stream (already running the next replay) is never blocked."""
        buf, rec = handle
        if self.side_stream is not None:
            with torch.cuda.stream(self.side_stream):
                self._finish(rec)
                return buf.cpu().numpy()
        self._finish(rec)
        return buf.numpy()

    def flush(self) -> None:
        while self._inflight:
            self._finish(self._inflight.popleft())
        while self._ctrl_sends:
            w, _ = self._ctrl_sends.popleft()
            w.wait()


def init_distributed(backend: Optional[str] = None, device: Optional[torch.device] = None):
    """Initialise torch.distributed from torchrun env vars (127.0.0.1 rendezvous).

    Failure detection: data-plane operations get a bounded timeout
    (``DLI_PP_TIMEOUT_S``, default 600 s), so a stage that dies mid-session turns a blocked
    exchange into an error: RCCL's watchdog aborts the communicator when the timeout fires
    (torch's ``TORCH_NCCL_ASYNC_ERROR_HANDLING`` default), gloo raises as soon as the dead
    peer's sockets close. The head then fails its pending requests and reports unhealthy
    (``worker/service.PipelineService``); the master's failure detector routes new requests
    to the remaining replicas."""
    if dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29511")
    if backend is None:
        backend = os.environ.get("DLI_DIST_BACKEND") or (
            "nccl" if torch.cuda.is_available() else "gloo")
    kw = {"timeout": timedelta(seconds=float(os.environ.get("DLI_PP_TIMEOUT_S", "600")))}
    if backend == "nccl" and device is not None:
        kw["device_id"] = device
    dist.init_process_group(backend=backend, **kw)
    return dist.get_rank(), dist.get_world_size()
