"""Dispatcher: queue consumers that route each request to a worker node.

Reference behaviour (``master/dashboard/views.py:305-455``): mark ``processing``; if loaded
``ModelShard`` rows exist for the model, POST ``/inference`` with ``shard_ids`` to the FIRST
node holding shards; otherwise POST ``/load_model`` (300 s) then ``/inference`` (120 s) to
the FIRST active node; write the result or the error. Same HTTP calls, payloads, timeouts
and error strings here, with these fixes:

* selection by placement then load: nodes whose loaded shards cover the model first,
  then the active node with the fewest requests in flight from this master (ties -> lowest
  id), instead of always the first node;
* a connection failure retries the request on the next candidate node (up to
  ``max_attempts``) and reports the node to the health monitor, instead of failing;
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
        """(nodes, shard_ids_by_node) — shard holders first, as in views.py:318-340."""
        shards = self.store.shards(model_name=model_name, loaded_only=True)
        if shards:
            by_node: Dict[int, List[int]] = defaultdict(list)
            for s in shards:
                by_node[s["node_id"]].append(s["shard_id"])
            nodes = [n for n in self.store.list_nodes(active_only=True) if n["id"] in by_node]
            return self._pick(nodes), by_node
        return self._pick(self.store.list_nodes(active_only=True)), None

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
            payload = {"model_name": model, "prompt": prompt, "max_length": self.max_length,
                       "timeout": WORKER_TIMEOUT}
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
        self.store.mark_failed(rid, f"Node returned status code {r.status_code}: {r.text}")
        return False, None

    def _forget(self, node_id: int) -> None:
        with self._lock:
            self._loaded = {k for k in self._loaded if k[0] != node_id}
