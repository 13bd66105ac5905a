"""Completion fan-out between the processes of one master (``serve-master --procs N``).

One Python master process tops out at ~550-600 requests/s (its GIL: two inbound HTTP
requests, one worker call and three store statements per generation, ~1.3 ms of CPU;
scripts/bench_control_plane.py). ``--procs N`` runs N copies of the ASGI master on the
same port (SO_REUSEPORT: the kernel spreads connections over them) and the same sqlite file.
Each process dispatches the requests it accepted (its own in-process queue), so a request's
whole life stays in one process — except its status long poll, which may arrive on any
connection, i.e. at any process. A process that finishes a request therefore sends its id
(8 bytes) to every peer over loopback UDP; a peer with long polls waiting on that id wakes
them, and they read the final row from the shared database. A lost datagram costs at most
the long poll's 2 s re-read (``Store.wait_final_async``). Rank 0 alone re-queues orphaned
requests at start and runs the node health monitor.
"""
from __future__ import annotations

import asyncio
import socket
import struct
from typing import Callable, List, Tuple

_FMT = "<q"


class PeerNotifier:
    def __init__(self, rank: int, nprocs: int, base_port: int):
        self.rank, self.nprocs, self.base_port = rank, nprocs, base_port
        self.peers: List[Tuple[str, int]] = [("127.0.0.1", base_port + i)
                                             for i in range(nprocs) if i != rank]
        self._sock = socket.socket(socket.AF_INET, socket.SOCK_DGRAM)
        self._sock.setblocking(False)
        self.sent = 0
        self.received = 0
        self._listening = False

    def publish(self, rid: int) -> None:
        """Tell every peer that request ``rid`` reached a final state (fire and forget)."""
        data = struct.pack(_FMT, int(rid))
        for p in self.peers:
            try:
                self._sock.sendto(data, p)
                self.sent += 1
            except OSError:          # full socket buffer: the peer's 2 s re-read covers it
                pass

    async def listen(self, on_final: Callable[[int], None]) -> None:
        """Receive peers' completions on this process's port (call once, on the server's
        event loop)."""
        if self._listening:
            return
        self._listening = True
        owner = self

        class _Proto(asyncio.DatagramProtocol):
            def datagram_received(self, data, addr):
                for (rid,) in struct.iter_unpack(_FMT, data[: len(data) - len(data) % 8]):
                    owner.received += 1
                    on_final(rid)

        loop = asyncio.get_running_loop()
        await loop.create_datagram_endpoint(
            _Proto, local_addr=("127.0.0.1", self.base_port + self.rank))
