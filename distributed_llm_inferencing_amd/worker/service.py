"""EngineService: one engine per loaded model, driven by a background thread.

The reference worker runs one sync gunicorn worker (``worker/Dockerfile:45``): every
``/inference`` call runs its own ``generate`` at batch 1 while others wait. Here HTTP handler
threads only enqueue; a single engine thread admits everything queued into the
continuous-batching scheduler and steps it, so concurrent requests share every decode step
(and every GEMM weight read).
"""
from __future__ import annotations

import contextlib
import queue
import threading
import time
from concurrent.futures import Future
from typing import Optional

from ..engine.sequence import SamplingParams


class EngineService:
    def __init__(self, engine, name: str = "engine"):
        self.engine = engine
        self.name = name
        self._inbox: "queue.Queue[tuple]" = queue.Queue()
        self._futures = {}
        self._stop = threading.Event()
        self._wake = threading.Event()
        self._ids = 0
        self._lock = threading.Lock()
        self.error: Optional[BaseException] = None
        self._t = threading.Thread(target=self._run, name=f"dli-engine-{name}", daemon=True)
        self._t.start()

    def submit(self, prompt, params: Optional[SamplingParams] = None) -> Future:
        fut: Future = Future()
        with self._lock:
            self._ids += 1
            rid = f"{self.name}-{self._ids}"
        self._inbox.put((rid, prompt, params, fut))
        self._wake.set()
        return fut

    def generate(self, prompt, params: Optional[SamplingParams] = None,
                 timeout: Optional[float] = None):
        return self.submit(prompt, params).result(timeout=timeout)

    def _admit(self):
        while True:
            try:
                rid, prompt, params, fut = self._inbox.get_nowait()
            except queue.Empty:
                return
            try:
                self.engine.add_request(prompt, params, request_id=rid)
                self._futures[rid] = fut
            except Exception as e:  # noqa: BLE001
                fut.set_exception(e)

    def _phase(self, name):
        t = getattr(self.engine, "timer", None)
        return t.phase(name) if t is not None else contextlib.nullcontext()

    def _run(self):
        while not self._stop.is_set():
            with self._phase("svc_admit"):
                self._admit()
            if not self.engine.has_work():
                self._wake.wait(0.05)
                self._wake.clear()
                continue
            try:
                outs = self.engine.step()
            except BaseException as e:  # noqa: BLE001 — fail every pending request loudly
                self.error = e
                for f in self._futures.values():
                    if not f.done():
                        f.set_exception(e)
                self._futures.clear()
                time.sleep(0.1)
                continue
            with self._phase("svc_resolve"):
                for o in outs:
                    f = self._futures.pop(o.request_id, None)
                    if f is not None and not f.done():
                        f.set_result(o)

    def stats(self) -> dict:
        s = self.engine.stats.snapshot() if hasattr(self.engine, "stats") else {}
        sch = getattr(self.engine, "scheduler", None)
        if sch is not None:
            s["prefix_hit_tokens"] = sch.prefix_hit_tokens
            s["preempted"] = sch.num_preempted
            s["max_seqs"] = sch.max_seqs
        bm = getattr(self.engine, "bm", None)
        if bm is not None:
            s["kv_free_blocks"] = bm.num_free
        if getattr(self.engine, "timer", None) is not None:
            s["phases"] = self.engine.timer.snapshot()     # host time per engine-loop phase
        s["queued"] = self._inbox.qsize()
        s["in_flight"] = len(self._futures)
        return s

    def close(self):
        self._stop.set()
        self._wake.set()
        self._t.join(5)


class PipelineFailed(RuntimeError):
    """The request's pipeline ring broke (a stage died): retryable on another replica."""


class PipelineService:
    """Same interface, backed by the rank-0 head of a DistributedPipelineEngine: a ring
    session runs while there is work, and requests join it at tick boundaries.

    A session that raises (a stage died, a link failed, the data-plane timeout fired) leaves
    the ring unusable: every pending and later request fails at once with that error, and
    ``error`` is set so the worker's /health and /inference answer 503 (the master's
    dispatcher re-sends the request to another replica, its failure detector takes the node
    out of rotation) instead of hanging requests on a broken ring. ``on_failure`` (the
    worker) then aborts the communicator; the process stays up and a new ``/load_shard``
    pipeline spec re-forms the ring with restarted or spare stage workers."""

    def __init__(self, pipe_engine, name: str = "pipeline", on_failure=None):
        self.engine = pipe_engine
        self.name = name
        self.on_failure = on_failure
        self._inbox: "queue.Queue[tuple]" = queue.Queue()
        self._stop = threading.Event()
        self._ids = 0
        self._lock = threading.Lock()
        self.error: Optional[BaseException] = None
        self._futs = {}
        self._carry = None               # the request that started a session, admitted first
        self.sessions = 0
        self._t = threading.Thread(target=self._run, name=f"dli-pipe-{name}", daemon=True)
        self._t.start()

    def submit(self, prompt, params=None) -> Future:
        fut: Future = Future()
        if self.error is not None:
            fut.set_exception(PipelineFailed(f"pipeline {self.name} failed: {self.error}"))
            return fut
        with self._lock:
            self._ids += 1
            rid = f"{self.name}-{self._ids}"
        self._inbox.put((rid, prompt, params, fut))
        return fut

    def _fail_pending(self):
        if self._carry is not None:
            self._carry[3].set_exception(PipelineFailed(f"pipeline {self.name} failed: {self.error}"))
            self._carry = None
        while True:
            try:
                _rid, _p, _s, fut = self._inbox.get_nowait()
            except queue.Empty:
                return
            fut.set_exception(PipelineFailed(f"pipeline {self.name} failed: {self.error}"))

    def generate(self, prompt, params=None, timeout=None):
        return self.submit(prompt, params).result(timeout=timeout)

    def _admit(self) -> int:
        """Tick boundary: move every queued request into the running head scheduler, in
        arrival order (the request that woke the session first)."""
        n = 0
        while True:
            if self._carry is not None:
                (rid, prompt, params, fut), self._carry = self._carry, None
            else:
                try:
                    rid, prompt, params, fut = self._inbox.get_nowait()
                except queue.Empty:
                    return n
            try:
                self.engine.add_request(prompt, params, request_id=rid)
                self._futs[rid] = fut
                n += 1
            except Exception as e:  # noqa: BLE001
                fut.set_exception(e)

    def _resolve(self, outs) -> None:
        for o in outs:
            f = self._futs.pop(o.request_id, None)
            if f is not None and not f.done():
                f.set_result(o)

    def _run(self):
        head = self.engine.head
        while not self._stop.is_set():
            try:
                self._carry = self._inbox.get(timeout=0.05)   # admitted by the first tick
            except queue.Empty:
                continue
            try:
                # continuous admission: requests that arrive while the ring is running join
                # it at the next tick; each finished request is answered the tick it finishes
                head.run_session(admit=self._admit, on_finished=self._resolve)
                self.sessions += 1
            except BaseException as e:  # noqa: BLE001 — the ring is broken: fail fast
                self.error = e
                err = PipelineFailed(f"pipeline {self.name} failed: {e}")
                for f in self._futs.values():
                    if not f.done():
                        f.set_exception(err)
                self._futs.clear()
                self._fail_pending()
                if self.on_failure is not None:
                    try:
                        self.on_failure(e)
                    except Exception:  # noqa: BLE001
                        pass
                return

    def stats(self) -> dict:
        s = self.engine.head.stats.snapshot()
        s["queued"] = self._inbox.qsize()
        s["failed"] = None if self.error is None else str(self.error)
        return s

    def close(self):
        self._stop.set()
        self._t.join(5)


class ExpertService:
    """Same interface, backed by one rank of an ExpertParallelEngine (``cli serve-expert``):
    every rank is a worker node of its own (DP attention, its own requests and KV) whose MoE
    layers exchange rows with the other ranks every step. The ranks step in lockstep, so
    this thread keeps stepping while ANY rank has work — an idle rank joins every exchange
    with an empty forward — and when none has, every rank sleeps on the group's shared
    doorbell (``ExpertParallelEngine.wait_bell``: a futex in the lockstep board) until a
    submit on any rank rings it, re-checking the group once every ``idle_s`` (no CPU while
    the group idles). ``close`` raises the stop bit of the exchange and rings: every rank
    leaves its loop once no rank has work, and requests still queued then fail ("group
    stopped"); submits after ``close`` fail at once. A failed exchange (a peer died) fails
    every pending request and sets ``error`` (the worker answers 503, the master's
    dispatcher retries on another node)."""

    def __init__(self, ep_engine, name: str = "expert", idle_s: float = 1.0):
        self.engine = ep_engine
        self.name = name
        self.idle_s = idle_s
        self._inbox: "queue.Queue[tuple]" = queue.Queue()
        self._futs = {}
        self._ids = 0
        self._lock = threading.Lock()
        self.error: Optional[BaseException] = None
        self.stopped = threading.Event()
        self._t = threading.Thread(target=self._run, name=f"dli-ep-{name}", daemon=True)
        self._t.start()

    def submit(self, prompt, params=None) -> Future:
        fut: Future = Future()
        ep = self.engine
        if (self.error is not None or self.stopped.is_set() or ep.stop_requested
                or ep.stopping):
            why = self.error if self.error is not None else "stopping"
            fut.set_exception(PipelineFailed(f"expert group {self.name} is down: {why}"))
            return fut
        with self._lock:
            self._ids += 1
            rid = f"{self.name}-r{self.engine.rank}-{self._ids}"
        self._inbox.put((rid, prompt, params, fut))
        ep.ring_bell()                      # wake the group if it sleeps
        return fut

    def generate(self, prompt, params=None, timeout=None):
        return self.submit(prompt, params).result(timeout=timeout)

    def _admit(self) -> None:
        eng = self.engine.engine
        while True:
            try:
                rid, prompt, params, fut = self._inbox.get_nowait()
            except queue.Empty:
                return
            try:
                eng.add_request(prompt, params, request_id=rid)
                self._futs[rid] = fut
            except Exception as e:  # noqa: BLE001
                fut.set_exception(e)

    def _fail_all(self, err: BaseException) -> None:
        exc = PipelineFailed(f"expert group {self.name} failed: {err}")
        for f in self._futs.values():
            if not f.done():
                f.set_exception(exc)
        self._futs.clear()
        while True:
            try:
                *_, fut = self._inbox.get_nowait()
            except queue.Empty:
                return
            fut.set_exception(exc)

    def _run(self):
        ep = self.engine
        self.idle_waits = 0
        try:
            while True:
                bell = ep.bell()                # read before looking for work (no lost ring)
                self._admit()
                outs, more = ep.step()
                for o in outs:
                    f = self._futs.pop(o.request_id, None)
                    if f is not None and not f.done():
                        f.set_result(o)
                if ep.stopping and not more:
                    break
                if not more and self._inbox.empty():
                    # every rank saw the same "no work": sleep until a submit on any rank
                    self.idle_waits += 1
                    ep.wait_bell(bell, self.idle_s)
            self._fail_all(RuntimeError("group stopped"))   # submits that raced the stop
        except BaseException as e:  # noqa: BLE001 — a peer died or the data plane broke
            self.error = e
            self._fail_all(e)
        finally:
            self.stopped.set()

    def stats(self) -> dict:
        s = self.engine.engine.stats.snapshot()
        s.update(queued=self._inbox.qsize(), in_flight=len(self._futs),
                 lockstep_steps=self.engine.steps, graph_steps=self.engine.graph_steps,
                 failed=None if self.error is None else str(self.error))
        return s

    def close(self, timeout: float = 30.0) -> None:
        """Ask the whole group to stop (collective: every rank's service leaves its loop)."""
        self.engine.stop_requested = True
        self.engine.ring_bell()
        self.stopped.wait(timeout)
