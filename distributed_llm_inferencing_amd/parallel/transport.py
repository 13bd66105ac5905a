"""Inter-stage transport for the layer-sharded pipeline.

The reference has NO inter-shard data plane (its "sharded" path runs shard 0 alone,
``worker/app.py:334-336``). Here a pipeline step moves over two planes:

* control plane (host): the head's packed ``StepMeta`` for every tick goes to every other
  stage over a separate **gloo** process group (TCP loopback, CPU tensors) the moment the
  head schedules it, so a stage's host can stage the metadata upload and enqueue its graph
  replay long before the activations arrive — no stage ever waits on its GPU to learn what
  to do next;
* data plane (device): hidden states stage r -> r+1 and sampled token ids tail -> head go by
  RCCL point-to-point over xGMI (``torch.distributed`` backend "nccl" == RCCL on ROCm),
  ordered on the GPU streams: the receive is a stream dependency of the consumer's graph
  replay, never a host wait. On CPU (tests) the data plane is gloo as well.

Every stage learns the activation shape of tick k from tick k's metadata (rows = tokens of
the step, cols = hidden size), so the data plane carries no headers at all. Sends and
receives between a pair of ranks are posted in the same (tick) order on both sides.
"""
from __future__ import annotations

import os
from collections import deque
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
    """Control + data planes of one pipeline rank (default process group = the stages)."""

    def __init__(self, device: torch.device, dtype=torch.bfloat16, max_pending: int = 8):
        self.rank = dist.get_rank()
        self.world = dist.get_world_size()
        self.device = torch.device(device)
        self.dtype = dtype
        self.nccl = dist.get_backend() == "nccl"
        # collective over all ranks, same order everywhere (called once per engine)
        self.ctrl_group = dist.new_group(backend="gloo")
        # one communicator per data edge (r -> r+1, and tail -> head): RCCL serialises the
        # operations of one communicator on one stream, so sharing a communicator would
        # queue the head's next send behind its wait for the tail's tokens
        edges = [dist.new_group([r, r + 1]) for r in range(self.world - 1)]
        ret = dist.new_group([0, self.world - 1]) if self.world > 1 else None
        self.out_group = (edges[self.rank] if self.rank < self.world - 1 else ret)
        self.in_group = edges[self.rank - 1] if self.rank > 0 else ret
        self.data_device = self.device if self.nccl else torch.device("cpu")
        self._sends = deque()
        self._ctrl_sends = deque()
        self.max_pending = max_pending
        self.recv_stream = (torch.cuda.Stream(self.device)
                            if self.nccl and self.device.type == "cuda" else None)

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
        while len(self._ctrl_sends) > 4 * self.world * 2:
            w, _ = self._ctrl_sends.popleft()
            w.wait()

    def recv_ctrl(self) -> Tuple[np.ndarray, np.ndarray]:
        h = torch.empty(HEADER_LEN, dtype=torch.int64)
        dist.recv(h, 0, group=self.ctrl_group)
        n = int(h[4])
        p = torch.empty(n, dtype=torch.int32)
        if n:
            dist.recv(p, 0, group=self.ctrl_group)
        return h.numpy(), p.numpy()

    # ------------------------------------------------------------------ data plane
    def send(self, t: torch.Tensor) -> None:
        """Asynchronous send of a snapshot of ``t`` (graph outputs are static buffers) to
        the next stage, or from the tail back to the head."""
        with trace_range("pp.send"):
            snap = t.clone() if self.nccl else t.to("cpu")
            w = dist.isend(snap.contiguous(), self.next, group=self.out_group)
            self._sends.append((w, snap))
        while len(self._sends) > self.max_pending:
            w, _ = self._sends.popleft()
            w.wait()

    def recv_hidden(self, rows: int, cols: int) -> torch.Tensor:
        """Receive stage input from the previous stage; on RCCL the wait is a stream
        dependency of the replay that consumes it, not a host wait."""
        with trace_range("pp.recv"):
            buf = torch.empty(rows, cols, dtype=self.dtype, device=self.data_device)
            dist.irecv(buf, self.prev, group=self.in_group).wait()
        return buf if buf.device == self.device else buf.to(self.device)

    def irecv_tokens(self, n: int):
        """Post the head's receive of a tick's sampled ids from the tail, on a side stream
        so the next replay does not depend on it (returns a handle)."""
        if self.recv_stream is not None:
            with torch.cuda.stream(self.recv_stream):
                buf = torch.empty(n, dtype=torch.int32, device=self.device)
                dist.irecv(buf, self.prev, group=self.in_group).wait()
            return buf, None
        buf = torch.empty(n, dtype=torch.int32)
        return buf, dist.irecv(buf, self.prev, group=self.in_group)

    def tokens_to_host(self, handle) -> np.ndarray:
        buf, work = handle
        if self.recv_stream is not None:
            with torch.cuda.stream(self.recv_stream):
                return buf.cpu().numpy()
        work.wait()
        return buf.numpy()

    def flush(self) -> None:
        while self._sends:
            w, _ = self._sends.popleft()
            w.wait()
        while self._ctrl_sends:
            w, _ = self._ctrl_sends.popleft()
            w.wait()


def init_distributed(backend: Optional[str] = None, device: Optional[torch.device] = None):
    """Initialise torch.distributed from torchrun env vars (127.0.0.1 rendezvous)."""
    if dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29511")
    if backend is None:
        backend = os.environ.get("DLI_DIST_BACKEND") or (
            "nccl" if torch.cuda.is_available() else "gloo")
    kw = {}
    if backend == "nccl" and device is not None:
        kw["device_id"] = device
    dist.init_process_group(backend=backend, **kw)
    return dist.get_rank(), dist.get_world_size()
