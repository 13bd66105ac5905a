"""Dispatcher: queue consumers that route each request to a worker node.

Reference behaviour (``master/dashboard/views.py:305-455``): mark ``processing``; if loaded
``ModelShard`` rows exist for the model, POST ``/inference`` with ``shard_ids`` to the FIRST
node holding shards; otherwise POST ``/load_model`` (300 s) then ``/inference`` (120 s) to
the FIRST active node; write the result or the error. Same HTTP calls, payloads, timeouts
and error strings here, with these fixes:

* selection by placement then load: nodes whose loaded shards cover the model first,
  then the active node with the fewest requests in flight from this master (ties -> lowest
  id), instead of always the first node;
* a connection failure, or a 503 from a node whose pipeline ring broke, retries the request
  on the next candidate node (up to ``max_attempts``: another replica) and reports the node
  to the health monitor, instead of failing (the reference fails over only at selection
  time, views.py:99-105,389-391);
* the worker's bearer token is sent when ``AUTH_KEY`` is configured (the reference never
  sends it, so enabling worker auth broke dispatch);
* a fixed pool of consumer threads instead of one unbounded thread per submit.
"""
from __future__ import annotations

import logging
import threading
import time
from collections import defaultdict
from typing import Callable, Dict, List, Optional

import requests

from ..utils import faults

log = logging.getLogger("dli.dispatcher")

MAX_LENGTH = 100            # views.py:351,417
WORKER_TIMEOUT = 60         # views.py:352,418 (cooperative compute timeout on the worker)
HTTP_INFER_TIMEOUT = 120    # views.py:354
HTTP_LOAD_TIMEOUT = 300     # views.py:400


class Dispatcher:
    def __init__(self, store, queue, settings, num_workers: int = 4, max_attempts: int = 3,
                 on_node_error: Optional[Callable[[int, str], None]] = None,
                 session: Optional[requests.Session] = None):
        self.store, self.queue, self.settings = store, queue, settings
        self.num_workers = num_workers
        self.max_attempts = max_attempts
        self.on_node_error = on_node_error
        self.http = session or requests.Session()
        if session is None:
            # one pooled keep-alive connection per consumer thread (urllib3 keeps 10 per
            # host by default: the rest were opened and discarded per request)
            ad = requests.adapters.HTTPAdapter(pool_connections=16,
                                               pool_maxsize=max(16, num_workers))
            self.http.mount("http://", ad)
            self.http.mount("https://", ad)
        self.inflight: Dict[int, int] = defaultdict(int)
        self._lock = threading.Lock()
        self._stop = threading.Event()
        self._threads: List[threading.Thread] = []
        self.max_length = MAX_LENGTH
        self.processed = 0
        # (node id, model) confirmed loaded: skip the /load_model round trip before every
        # /inference (the reference posts it each time, views.py:397-401; the worker also
        # auto-loads on /inference, app.py:278-282). Dropped on any error from that node.
        self._loaded: set = set()
        self.load_calls = 0
        self._cand_cache: Dict[str, tuple] = {}

    # ------------------------------------------------------------------ lifecycle
    def start(self):
        for i in range(self.num_workers):
            t = threading.Thread(target=self._loop, name=f"dli-dispatch-{i}", daemon=True)
            t.start()
            self._threads.append(t)

    def stop(self, timeout: float = 5.0):
        self._stop.set()
        for t in self._threads:
            t.join(timeout)

    def submit(self, request_id: int):
        self.queue.put(request_id)

    def _loop(self):
        while not self._stop.is_set():
            rid = self.queue.get(timeout=0.2)
            if rid is None:
                continue
            try:
                self.process(rid)
            finally:
                rel = getattr(self.queue, "release", None)
                if rel:
                    rel(rid)

    # ------------------------------------------------------------------ helpers
    def _headers(self) -> dict:
        if self.settings.auth_key:
            return {"Authorization": f"Bearer {self.settings.auth_key}"}
        return {}

    def _pick(self, nodes: List[dict]) -> List[dict]:
        with self._lock:
            return sorted(nodes, key=lambda n: (self.inflight[n["id"]], n["id"]))

    def _post(self, node: dict, path: str, payload: dict, timeout: float):
        return self.http.post(f"{node['url']}{path}", json=payload, timeout=timeout,
                              headers=self._headers())

    def _candidates(self, model_name: str):
        """(nodes, shard_ids_by_node) — shard holders first, as in views.py:318-340. The
        node / shard rows are re-read when this process changed them (store topology
        version) or after 0.5 s (another process, the heartbeat of a shared database): per-
        request reads contended the store lock at hundreds of requests/s; the load order is
        recomputed every time."""
        now = time.monotonic()
        ver = getattr(self.store, "topology_version", 0)
        hit = self._cand_cache.get(model_name)
        if hit is None or now - hit[0] > 0.5 or hit[1] != ver:
            hit = (now, ver, self._candidates_uncached(model_name))
            self._cand_cache[model_name] = hit
        nodes, by_node = hit[2]
        return self._pick(nodes), by_node

    def invalidate_candidates(self) -> None:
        self._cand_cache.clear()

    def _candidates_uncached(self, model_name: str):
        shards = self.store.shards(model_name=model_name, loaded_only=True)
        if shards:
            by_node: Dict[int, List[int]] = defaultdict(list)
            for s in shards:
                by_node[s["node_id"]].append(s["shard_id"])
            nodes = [n for n in self.store.list_nodes(active_only=True) if n["id"] in by_node]
            return nodes, by_node
        return self.store.list_nodes(active_only=True), None

    # ------------------------------------------------------------------ the request path
    def process(self, rid: int) -> None:
        try:
            req = self.store.get_request(rid)
        except KeyError:
            return
        model, prompt = req["model_name"], req["prompt"]
        try:
            nodes, shard_map = self._candidates(model)
            if not nodes:
                self.store.mark_processing(rid)
                self.store.mark_failed(rid, "No active nodes with loaded shards found"
                                       if shard_map is not None else
                                       "No active worker nodes available")
                return
            last_err = None
            for node in nodes[: self.max_attempts]:
                self.store.mark_processing(rid, node["id"])
                with self._lock:
                    self.inflight[node["id"]] += 1
                try:
                    ok, err = self._run_on(node, rid, model, prompt,
                                           shard_map[node["id"]] if shard_map else None)
                finally:
                    with self._lock:
                        self.inflight[node["id"]] -= 1
                if ok:
                    return
                if err is None:        # terminal (worker answered with an error) — recorded
                    return
                last_err = err         # connection-level: try the next node
                if self.on_node_error:
                    self.on_node_error(node["id"], err)
            self.store.mark_failed(rid, last_err or "all candidate nodes failed")
        except Exception as e:  # noqa: BLE001 — views.py:445-455 fatal fallback
            log.critical("Fatal error processing inference request %s: %s", rid, e)
            try:
                self.store.mark_failed(rid, f"Fatal error: {e}")
            except Exception:  # noqa: BLE001
                pass
        finally:
            self.processed += 1

    def _run_on(self, node, rid, model, prompt, shard_ids):
        """Returns (True, None) on success, (False, None) on a recorded terminal failure,
        (False, msg) on a connection failure (retry elsewhere)."""
        t0 = time.perf_counter()
        try:
            faults.check("dispatch.post")
            if shard_ids is None and (node["id"], model) not in self._loaded:
                self.load_calls += 1
                r = self._post(node, "/load_model", {"model_name": model}, HTTP_LOAD_TIMEOUT)
                if r.status_code != 200:
                    self.store.mark_failed(rid, f"Failed to load model: {r.text}")
                    return False, None
                with self._lock:
                    self._loaded.add((node["id"], model))
            # seed = this master's request id: the sampled tokens of a request do not depend
            # on which node (or which retry) serves it
            payload = {"model_name": model, "prompt": prompt, "max_length": self.max_length,
                       "timeout": WORKER_TIMEOUT, "seed": int(rid)}
            if shard_ids is not None:
                payload["shard_ids"] = sorted(shard_ids)
            r = self._post(node, "/inference", payload, HTTP_INFER_TIMEOUT)
        except (requests.RequestException, faults.InjectedFault) as e:
            self._forget(node["id"])
            return False, f"Connection error: {e}"
        if r.status_code == 200:
            data = r.json()
            if data.get("status") == "success":
                self.store.mark_completed(rid, data.get("result", ""),
                                          data.get("execution_time", time.perf_counter() - t0))
                return True, None
            self.store.mark_failed(rid, data.get("message", "Unknown error"))
            return False, None
        self._forget(node["id"])
        if r.status_code == 503:               # the node's pipeline broke: next replica
            return False, f"Node returned status code 503: {r.text[:300]}"
        self.store.mark_failed(rid, f"Node returned status code {r.status_code}: {r.text}")
        return False, None

    def _forget(self, node_id: int) -> None:
        with self._lock:
            self._loaded = {k for k in self._loaded if k[0] != node_id}


class AsyncDispatcher(Dispatcher):
    """The same request path on ONE asyncio event loop (aiohttp) instead of one blocked
    thread per in-flight request.

    Each in-flight request holds its dispatcher thread for the whole generation (0.3-3 s)
    in the threaded design; at 512 requests in flight that is 512 CPython threads plus the
    HTTP server's, and the master topped out at ~130 requests/s with the GIL handing itself
    around (~45 % of one core busy, most threads waiting to be scheduled). Here every worker
    call is a coroutine on one loop; ``num_workers`` bounds the calls in flight (same
    meaning as the thread count). Node selection, retries, load caching, messages and
    timeouts are those of ``Dispatcher``."""

    def start(self):
        import asyncio
        self._loop = asyncio.new_event_loop()
        self._done = threading.Event()
        t = threading.Thread(target=self._loop_main, name="dli-dispatch-aio", daemon=True)
        t.start()
        self._threads.append(t)

    def start_on_loop(self, loop) -> None:
        """Run the dispatch loop as a task on ``loop`` (the ASGI server's own event loop)
        instead of a thread of its own: the submit handler, the long polls and the worker
        calls then share one thread, so a request never crosses threads on its hot path
        (no self-pipe wake-ups, no GIL hand-offs; the inline store's lock is uncontended)."""
        if getattr(self, "_task", None) is not None or self._threads:
            return
        import asyncio
        self._loop = loop
        self._wake = asyncio.Event()
        self._task = loop.create_task(self._main())

    def submit(self, request_id: int):
        self.queue.put(request_id)
        wake = getattr(self, "_wake", None)
        if wake is not None:                 # on-loop mode: wake the dispatch loop now
            import asyncio
            try:
                here = asyncio.get_running_loop()
            except RuntimeError:
                here = None
            if here is self._loop:
                wake.set()
            else:
                self._loop.call_soon_threadsafe(wake.set)

    def stop(self, timeout: float = 5.0):
        self._stop.set()
        for t in self._threads:
            t.join(timeout)

    def _loop_main(self):
        import asyncio
        asyncio.set_event_loop(self._loop)
        try:
            self._loop.run_until_complete(self._main())
        finally:
            self._loop.close()

    async def _main(self):
        import asyncio
        from concurrent.futures import ThreadPoolExecutor

        import aiohttp
        loop = asyncio.get_running_loop()
        self._session = aiohttp.ClientSession(connector=aiohttp.TCPConnector(limit=0))
        sem = asyncio.Semaphore(max(1, self.num_workers))
        getter = ThreadPoolExecutor(1, thread_name_prefix="dli-dispatch-q")
        # store calls wait on the store's database thread: run them off the loop, several at
        # once, so the database thread can batch them into one transaction
        self._dbpool = ThreadPoolExecutor(32, thread_name_prefix="dli-dispatch-db")
        tasks = set()
        try:
            while not self._stop.is_set():
                await sem.acquire()
                free = 1
                while free < 256 and not sem.locked():     # claim every free slot (burst)
                    await sem.acquire()
                    free += 1
                wake = getattr(self, "_wake", None)
                if wake is not None and getattr(self.queue, "name", "") == "inproc":
                    # on the server's loop: take what is queued without a thread hop; when
                    # nothing is, sleep until a submit wakes us (or 0.2 s, for producers in
                    # other processes: the sqlite / redis queues)
                    rids = self.queue.get_many(free, 0.0)
                    if not rids:
                        wake.clear()
                        rids = self.queue.get_many(free, 0.0)   # a submit raced the clear
                    if not rids:
                        for _ in range(free):
                            sem.release()
                        try:
                            await asyncio.wait_for(wake.wait(), 0.2)
                        except asyncio.TimeoutError:
                            pass
                        continue
                else:
                    rids = await loop.run_in_executor(getter, self.queue.get_many, free, 0.2)
                for _ in range(free - len(rids)):
                    sem.release()
                for rid in rids:
                    t = asyncio.create_task(self._process_async(rid, sem))
                    tasks.add(t)
                    t.add_done_callback(tasks.discard)
        finally:
            for t in list(tasks):
                t.cancel()
            await asyncio.gather(*tasks, return_exceptions=True)
            await self._session.close()
            getter.shutdown(wait=False)
            self._dbpool.shutdown(wait=False)

    async def _s(self, fn, *args):
        """A store call, awaited without blocking the event loop: run on the store's database
        thread itself when the store offers it (no thread hop), else on a small pool."""
        import asyncio
        if getattr(self.store, "inline", False):
            return fn(*args)                     # the caller's thread runs the statement
        submit = getattr(self.store, "submit", None)
        if submit is not None:
            return await asyncio.wrap_future(submit(lambda _c: fn(*args)))
        return await asyncio.get_running_loop().run_in_executor(self._dbpool, fn, *args)

    async def _process_async(self, rid: int, sem) -> None:
        try:
            await self.process_async(rid)
        finally:
            sem.release()
            rel = getattr(self.queue, "release", None)
            if rel:
                rel(rid)

    async def process_async(self, rid: int) -> None:
        mark = getattr(self.store, "mark_time", None)
        if mark is not None:
            mark(rid, 1)
        try:
            fields = getattr(self.store, "request_fields", None)
            if fields is not None:
                model, prompt = await self._s(fields, rid)
            else:
                req = await self._s(self.store.get_request, rid)
                model, prompt = req["model_name"], req["prompt"]
        except KeyError:
            return
        try:
            nodes, shard_map = await self._s(self._candidates, model)
            if not nodes:
                await self._s(self.store.mark_processing, rid)
                await self._s(self.store.mark_failed, rid, "No active nodes with loaded shards found"
                                       if shard_map is not None else
                                       "No active worker nodes available")
                return
            last_err = None
            for node in nodes[: self.max_attempts]:
                await self._s(self.store.mark_processing, rid, node["id"])
                with self._lock:
                    self.inflight[node["id"]] += 1
                try:
                    ok, err = await self._run_on_async(
                        node, rid, model, prompt, shard_map[node["id"]] if shard_map else None)
                finally:
                    with self._lock:
                        self.inflight[node["id"]] -= 1
                if ok or err is None:
                    return
                last_err = err
                if self.on_node_error:
                    self.on_node_error(node["id"], err)
            await self._s(self.store.mark_failed, rid, last_err or "all candidate nodes failed")
        except Exception as e:  # noqa: BLE001 — views.py:445-455 fatal fallback
            log.critical("Fatal error processing inference request %s: %s", rid, e)
            try:
                await self._s(self.store.mark_failed, rid, f"Fatal error: {e}")
            except Exception:  # noqa: BLE001
                pass
        finally:
            self.processed += 1

    async def _post_async(self, node, path, payload, timeout):
        import aiohttp
        async with self._session.post(f"{node['url']}{path}", json=payload,
                                      headers=self._headers(),
                                      timeout=aiohttp.ClientTimeout(total=timeout)) as r:
            return r.status, await r.text()

    async def _run_on_async(self, node, rid, model, prompt, shard_ids):
        import asyncio
        import json as _json

        import aiohttp
        t0 = time.perf_counter()
        try:
            faults.check("dispatch.post")
            if shard_ids is None and (node["id"], model) not in self._loaded:
                self.load_calls += 1
                st, text = await self._post_async(node, "/load_model", {"model_name": model},
                                                  HTTP_LOAD_TIMEOUT)
                if st != 200:
                    await self._s(self.store.mark_failed, rid, f"Failed to load model: {text}")
                    return False, None
                with self._lock:
                    self._loaded.add((node["id"], model))
            # seed = this master's request id: the sampled tokens of a request do not depend
            # on which node (or which retry) serves it
            payload = {"model_name": model, "prompt": prompt, "max_length": self.max_length,
                       "timeout": WORKER_TIMEOUT, "seed": int(rid)}
            if shard_ids is not None:
                payload["shard_ids"] = sorted(shard_ids)
            st, text = await self._post_async(node, "/inference", payload, HTTP_INFER_TIMEOUT)
            mark = getattr(self.store, "mark_time", None)
            if mark is not None:
                mark(rid, 2)
        except (aiohttp.ClientError, asyncio.TimeoutError, OSError,
                faults.InjectedFault) as e:
            self._forget(node["id"])
            return False, f"Connection error: {e}"
        if st == 200:
            data = _json.loads(text)
            if data.get("status") == "success":
                await self._s(self.store.mark_completed, rid, data.get("result", ""),
                              data.get("execution_time", time.perf_counter() - t0))
                return True, None
            await self._s(self.store.mark_failed, rid, data.get("message", "Unknown error"))
            return False, None
        self._forget(node["id"])
        if st == 503:                          # the node's pipeline broke: next replica
            return False, f"Node returned status code 503: {text[:300]}"
        await self._s(self.store.mark_failed, rid, f"Node returned status code {st}: {text}")
        return False, None


def make_dispatcher(store, queue, settings, **kw) -> Dispatcher:
    """The asyncio dispatcher when aiohttp is importable (``DLI_DISPATCH=threads`` forces
    the thread pool)."""
    import os
    if os.environ.get("DLI_DISPATCH", "async") != "threads":
        try:
            import aiohttp  # noqa: F401
            return AsyncDispatcher(store, queue, settings, **kw)
        except ImportError:
            pass
    return Dispatcher(store, queue, settings, **kw)
