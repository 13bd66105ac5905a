"""Request queue with Redis-compatible semantics.

The reference configures Redis (``settings.py:95-97``, ``docker-compose.yml:57-63``) but
never uses it: every submit spawns an unbounded ``threading.Thread`` (``views.py:233``).
Here submits enqueue request ids and a fixed pool of dispatcher consumers drains the queue.

Backends (``QUEUE_BACKEND``):
    inproc  ``queue.Queue`` (default; single master process)
    sqlite  the ``pending`` rows of inference_request ARE the queue (survives restarts,
            shareable between master processes on one host)
    redis   LPUSH / BRPOP on a list, only if the ``redis`` client is importable
"""
from __future__ import annotations

import queue as _q
import threading
import time
from typing import Optional


class RequestQueue:
    name = "base"

    def put(self, request_id: int) -> None:
        raise NotImplementedError

    def get(self, timeout: float = 1.0) -> Optional[int]:
        raise NotImplementedError

    def get_many(self, max_n: int, timeout: float = 1.0) -> list:
        """Up to ``max_n`` ids: waits for the first, then takes what is already queued (the
        asyncio dispatcher drains a burst per hop to its loop)."""
        first = self.get(timeout)
        if first is None:
            return []
        out = [first]
        while len(out) < max_n:
            nxt = self.get(0.0)
            if nxt is None:
                break
            out.append(nxt)
        return out

    def qsize(self) -> int:
        return 0

    def close(self) -> None:
        pass


class InProcQueue(RequestQueue):
    name = "inproc"

    def __init__(self):
        self._q: _q.Queue = _q.Queue()

    def put(self, request_id: int) -> None:
        self._q.put(int(request_id))

    def get(self, timeout: float = 1.0) -> Optional[int]:
        try:
            if timeout <= 0:
                return self._q.get_nowait()
            return self._q.get(timeout=timeout)
        except _q.Empty:
            return None

    def qsize(self) -> int:
        return self._q.qsize()


class SqliteQueue(RequestQueue):
    """Claims the oldest pending request id not yet handed out by this process."""
    name = "sqlite"

    def __init__(self, store, poll_s: float = 0.05):
        self.store = store
        self.poll_s = poll_s
        self._claimed = set()
        self._lock = threading.Lock()
        self._event = threading.Event()

    def put(self, request_id: int) -> None:
        self._event.set()

    def get(self, timeout: float = 1.0) -> Optional[int]:
        deadline = time.monotonic() + timeout
        while True:
            with self._lock:
                for rid in self.store.pending_ids():
                    if rid not in self._claimed:
                        self._claimed.add(rid)
                        return rid
            left = deadline - time.monotonic()
            if left <= 0:
                return None
            self._event.wait(min(self.poll_s, left))
            self._event.clear()

    def release(self, request_id: int) -> None:
        with self._lock:
            self._claimed.discard(request_id)

    def qsize(self) -> int:
        return len([r for r in self.store.pending_ids() if r not in self._claimed])


class RedisQueue(RequestQueue):
    name = "redis"

    def __init__(self, host: str, port: int, db: int, key: str = "dli:requests"):
        import redis  # noqa: F401  (not installed in this image; optional)
        self._r = redis.Redis(host=host, port=port, db=db)
        self.key = key

    def put(self, request_id: int) -> None:
        self._r.lpush(self.key, int(request_id))

    def get(self, timeout: float = 1.0) -> Optional[int]:
        item = self._r.brpop(self.key, timeout=max(1, int(timeout)))
        return None if item is None else int(item[1])

    def qsize(self) -> int:
        return int(self._r.llen(self.key))


def make_queue(backend: str, store=None, settings=None) -> RequestQueue:
    backend = (backend or "inproc").lower()
    if backend == "sqlite":
        return SqliteQueue(store)
    if backend == "redis":
        try:
            return RedisQueue(settings.redis_host, settings.redis_port, settings.redis_db)
        except ImportError:
            return InProcQueue()      # redis client unavailable: degrade, never crash
    return InProcQueue()
