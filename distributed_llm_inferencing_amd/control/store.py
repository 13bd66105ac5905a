"""Control-plane state: sqlite3 store with the reference's three tables.

Mirrors the Django models of the reference (``master/dashboard/models.py:4-62``):

* worker_node    (id, hostname, ip_address, port=5000, is_active=False, last_heartbeat,
                  created_at, updated_at) + get_url() -> http://{ip}:{port}
* model_shard    (id, node_id -> worker_node ON DELETE CASCADE, model_name, shard_id,
                  is_loaded=False, created_at, updated_at), UNIQUE(model_name, shard_id)
* inference_request (id, model_name, prompt, result, error,
                  status in {pending, processing, completed, failed}, created_at, completed_at)
                  with mark_completed / mark_failed.

The reference has no migrations directory, so its tables would not exist
after ``migrate``; here the schema is created on startup. One database thread owns the
connection and serialises every access (the reference mutated sqlite from unbounded
threads, §5.2).
Extensions: node ``resources``/``gpu_id``/``role`` columns, request timing + node columns,
and ``recover()`` which re-queues requests orphaned in ``processing`` by a restart (§5.4).
"""
from __future__ import annotations

import json
import os
import queue
import sqlite3
import threading
import time
from datetime import datetime, timezone
from typing import Any, Dict, List, Optional

STATUSES = ("pending", "processing", "completed", "failed")

_SCHEMA = """
CREATE TABLE IF NOT EXISTS worker_node (
    id INTEGER PRIMARY KEY AUTOINCREMENT,
    hostname TEXT NOT NULL,
    ip_address TEXT NOT NULL,
    port INTEGER NOT NULL DEFAULT 5000,
    is_active INTEGER NOT NULL DEFAULT 0,
    last_heartbeat TEXT,
    created_at TEXT NOT NULL,
    updated_at TEXT NOT NULL,
    resources TEXT,
    failures INTEGER NOT NULL DEFAULT 0
);
CREATE TABLE IF NOT EXISTS model_shard (
    id INTEGER PRIMARY KEY AUTOINCREMENT,
    node_id INTEGER NOT NULL REFERENCES worker_node(id) ON DELETE CASCADE,
    model_name TEXT NOT NULL,
    shard_id INTEGER NOT NULL,
    is_loaded INTEGER NOT NULL DEFAULT 0,
    path TEXT,
    created_at TEXT NOT NULL,
    updated_at TEXT NOT NULL,
    UNIQUE(model_name, shard_id)
);
CREATE TABLE IF NOT EXISTS inference_request (
    id INTEGER PRIMARY KEY AUTOINCREMENT,
    model_name TEXT NOT NULL,
    prompt TEXT NOT NULL,
    result TEXT,
    error TEXT,
    status TEXT NOT NULL DEFAULT 'pending',
    created_at TEXT NOT NULL,
    completed_at TEXT,
    started_at TEXT,
    node_id INTEGER,
    attempts INTEGER NOT NULL DEFAULT 0,
    execution_time REAL
);
CREATE INDEX IF NOT EXISTS ix_req_status ON inference_request(status);
CREATE INDEX IF NOT EXISTS ix_req_created ON inference_request(created_at);
"""


def now_iso() -> str:
    return datetime.now(timezone.utc).isoformat()


class NotFound(KeyError):
    pass


class _Call:
    __slots__ = ("fn", "ev", "result", "error", "fut")

    def __init__(self, fn, fut=None):
        self.fn, self.ev, self.result, self.error = fn, threading.Event(), None, None
        self.fut = fut                      # concurrent.futures.Future for async callers


class _Exec:
    __slots__ = ("lastrowid", "rowcount")

    def __init__(self, cur):
        self.lastrowid, self.rowcount = cur.lastrowid, cur.rowcount


class Store:
    """Two access modes (``inline``, below). Inline (default): the caller runs its call
    under one re-entrant lock; with the threaded WSGI server's hundreds of threads that lock
    convoyed on the GIL (~140 requests/s), but the ASGI fronts run the hot path on ONE event
    loop (plus the async dispatcher's), so the lock is almost never contended. Threaded
    (``DLI_STORE_INLINE=0``): ONE database thread owns the connection; every other thread
    hands it a call and sleeps until it is done, and the thread runs the calls queued
    meanwhile in one transaction (one commit per batch) — the better mode for the
    thread-per-request werkzeug server."""

    def __init__(self, path: str = ":memory:", inline: Optional[bool] = None):
        self.path = path
        # inline mode (DLI_STORE_INLINE=1, default): calls run on the CALLER's thread under one
        # re-entrant lock, one commit per outermost call. The asyncio hot path (ASGI submit,
        # async dispatcher) then never hands a statement to another thread: with the
        # database thread, every sqlite3 call released the GIL and waited for it to come back
        # from the busy event loop (~0.5 ms wall per statement, cProfile of the master at
        # ~400 requests/s, scripts/bench_control_plane.py), which serialised the dispatcher.
        self.inline = (os.environ.get("DLI_STORE_INLINE", "1") == "1"
                       if inline is None else bool(inline))
        self._waiters: Dict[int, threading.Event] = {}   # long polls, by request id
        self._awaiters: Dict[int, list] = {}             # asyncio long polls: [(loop, fut)]
        self._wlock = threading.Lock()
        # rows of requests in a TERMINAL state (completed / failed never change again, so
        # the copy cannot go stale even when other processes share the database): status
        # reads of finished requests skip the database
        self._final_rows: Dict[int, Dict[str, Any]] = {}
        # rows of requests THIS process created and has not seen finish: the dispatcher
        # reads their (immutable) model / prompt and a long poll its first answer from here
        # instead of a SELECT each (other processes sharing the database are still seen:
        # a long poll re-reads the row every 2 s)
        self._live_rows: Dict[int, Dict[str, Any]] = {}
        self._returning = sqlite3.sqlite_version_info >= (3, 35, 0)
        # control-plane latency of requests created here: [submitted, dispatched, worker
        # answered] (perf_counter), folded into cp_timing when the long poll answers
        self._tmarks: Dict[int, list] = {}
        self.cp_timing = {"answered": 0, "queue_s": 0.0, "worker_s": 0.0, "answer_s": 0.0}
        # called with a request id when this process finished it (peer fan-out, peers.py)
        self.on_final = None
        self.topology_version = 0
        self._q: "queue.SimpleQueue[_Call]" = queue.SimpleQueue()
        self._conn_obj: Optional[sqlite3.Connection] = None
        if self.inline:
            self._ilock = threading.RLock()
            self._depth = 0
            self._conn_obj = self._connect()
        else:
            ready = threading.Event()
            self._t = threading.Thread(target=self._run, args=(ready,), name="dli-store",
                                       daemon=True)
            self._t.start()
            ready.wait()
        self._call(lambda c: c.executescript(_SCHEMA))

    def _connect(self) -> sqlite3.Connection:
        # File databases run in WAL mode with synchronous=NORMAL (a commit appends to the
        # WAL without an fsync); other processes (a second master worker, the sqlite queue)
        # share the file safely.
        c = sqlite3.connect(self.path, timeout=30, check_same_thread=False)
        c.row_factory = sqlite3.Row
        c.execute("PRAGMA foreign_keys = ON")
        if self.path != ":memory:":
            c.execute("PRAGMA journal_mode = WAL")
            c.execute("PRAGMA synchronous = NORMAL")
        return c

    # ------------------------------------------------------------------ the db thread
    def _run(self, ready: threading.Event):
        c = self._connect()
        self._conn_obj = c
        self._tid = threading.get_ident()
        ready.set()
        while True:
            batch = [self._q.get()]
            while len(batch) < 256:
                try:
                    batch.append(self._q.get_nowait())
                except queue.Empty:
                    break
            for call in batch:
                try:
                    call.result = call.fn(c)
                except BaseException as e:  # noqa: BLE001 — returned to the caller
                    call.error = e
            try:
                c.commit()
            except sqlite3.Error as e:
                for call in batch:
                    call.error = call.error or e
            for call in batch:
                if call.fut is not None:
                    if call.error is not None:
                        call.fut.set_exception(call.error)
                    else:
                        call.fut.set_result(call.result)
                call.ev.set()

    def _call(self, fn):
        if self.inline:
            with self._ilock:
                self._depth += 1
                try:
                    r = fn(self._conn_obj)
                    if self._depth == 1:
                        self._conn_obj.commit()
                    return r
                except BaseException:
                    if self._depth == 1:
                        self._conn_obj.rollback()
                    raise
                finally:
                    self._depth -= 1
        if threading.get_ident() == getattr(self, "_tid", None):
            return fn(self._conn_obj)                     # nested call on the db thread
        call = _Call(fn)
        self._q.put(call)
        call.ev.wait()
        if call.error is not None:
            raise call.error
        return call.result

    def submit(self, fn) -> "concurrent.futures.Future":
        """Run fn(connection) on the database thread; returns a Future (asyncio callers
        await it with ``asyncio.wrap_future`` instead of blocking a thread)."""
        import concurrent.futures
        fut: concurrent.futures.Future = concurrent.futures.Future()
        if self.inline:                        # run now, on this thread: a done future
            try:
                fut.set_result(self._call(fn))
            except BaseException as e:  # noqa: BLE001 — delivered through the future
                fut.set_exception(e)
            return fut
        self._q.put(_Call(fn, fut))
        return fut

    def _exec(self, sql: str, args=()):
        def run(c):
            r = _Exec(c.execute(sql, args))
            if "worker_node" in sql or "model_shard" in sql:
                self.topology_version += 1           # node / shard rows changed
            return r
        return self._call(run)

    def _query(self, sql: str, args=()) -> List[Dict[str, Any]]:
        return self._call(lambda c: [dict(r) for r in c.execute(sql, args).fetchall()])

    # ------------------------------------------------------------------ nodes
    def add_node(self, hostname: str, ip_address: str, port: int = 5000, is_active=False,
                 last_heartbeat: Optional[str] = None) -> int:
        t = now_iso()
        cur = self._exec("INSERT INTO worker_node (hostname, ip_address, port, is_active, "
                         "last_heartbeat, created_at, updated_at) VALUES (?,?,?,?,?,?,?)",
                         (hostname, ip_address, int(port), int(bool(is_active)), last_heartbeat,
                          t, t))
        return int(cur.lastrowid)

    def get_node(self, node_id: int) -> Dict[str, Any]:
        rows = self._query("SELECT * FROM worker_node WHERE id=?", (node_id,))
        if not rows:
            raise NotFound(f"No WorkerNode matches the given query (id={node_id}).")
        return self._node(rows[0])

    def list_nodes(self, active_only: bool = False) -> List[Dict[str, Any]]:
        q = "SELECT * FROM worker_node" + (" WHERE is_active=1" if active_only else "")
        return [self._node(r) for r in self._query(q + " ORDER BY id")]

    @staticmethod
    def _node(r: dict) -> dict:
        r["is_active"] = bool(r["is_active"])
        r["resources"] = json.loads(r["resources"]) if r.get("resources") else None
        r["url"] = f"http://{r['ip_address']}:{r['port']}"
        return r

    def update_node(self, node_id: int, **fields):
        if not fields:
            return
        if "resources" in fields and not isinstance(fields["resources"], (str, type(None))):
            fields["resources"] = json.dumps(fields["resources"])
        if "is_active" in fields:
            fields["is_active"] = int(bool(fields["is_active"]))
        fields["updated_at"] = now_iso()
        cols = ", ".join(f"{k}=?" for k in fields)
        self._exec(f"UPDATE worker_node SET {cols} WHERE id=?", (*fields.values(), node_id))

    def delete_node(self, node_id: int):
        self.get_node(node_id)
        self._exec("DELETE FROM worker_node WHERE id=?", (node_id,))

    def count_nodes(self, active_only=False) -> int:
        q = "SELECT COUNT(*) AS n FROM worker_node" + (" WHERE is_active=1" if active_only else "")
        return int(self._query(q)[0]["n"])

    # ------------------------------------------------------------------ shards
    def add_shard(self, node_id: int, model_name: str, shard_id: int, is_loaded=False,
                  path: Optional[str] = None) -> int:
        t = now_iso()

        def tx(_c):
            existing = self._query("SELECT id FROM model_shard WHERE model_name=? AND shard_id=?",
                                   (model_name, shard_id))
            if existing:
                self._exec("UPDATE model_shard SET node_id=?, is_loaded=?, path=?, updated_at=? "
                           "WHERE id=?", (node_id, int(bool(is_loaded)), path, t,
                                          existing[0]["id"]))
                return int(existing[0]["id"])
            cur = self._exec("INSERT INTO model_shard (node_id, model_name, shard_id, is_loaded, "
                             "path, created_at, updated_at) VALUES (?,?,?,?,?,?,?)",
                             (node_id, model_name, int(shard_id), int(bool(is_loaded)), path, t, t))
            return int(cur.lastrowid)
        return self._call(tx)

    def shards(self, model_name: Optional[str] = None, node_id: Optional[int] = None,
               loaded_only: bool = False) -> List[Dict[str, Any]]:
        q, a = "SELECT * FROM model_shard WHERE 1=1", []
        if model_name is not None:
            q += " AND model_name=?"
            a.append(model_name)
        if node_id is not None:
            q += " AND node_id=?"
            a.append(node_id)
        if loaded_only:
            q += " AND is_loaded=1"
        rows = self._query(q + " ORDER BY model_name, shard_id", a)
        for r in rows:
            r["is_loaded"] = bool(r["is_loaded"])
        return rows

    def delete_shard(self, shard_pk: int):
        self._exec("DELETE FROM model_shard WHERE id=?", (shard_pk,))

    # ------------------------------------------------------------------ requests
    def create_request(self, model_name: str, prompt: str) -> int:
        t = now_iso()
        cur = self._exec("INSERT INTO inference_request (model_name, prompt, status, created_at)"
                         " VALUES (?,?, 'pending', ?)", (model_name, prompt, t))
        rid = int(cur.lastrowid)
        if len(self._live_rows) > 200_000:            # bounded: drop the oldest half
            for k in sorted(self._live_rows)[:100_000]:
                self._live_rows.pop(k, None)
        if len(self._tmarks) > 200_000:
            self._tmarks.clear()
        self._tmarks[rid] = [time.perf_counter(), 0.0, 0.0]
        self._live_rows[rid] = {"id": rid, "model_name": model_name, "prompt": prompt,
                                "result": None, "error": None, "status": "pending",
                                "created_at": t, "completed_at": None, "started_at": None,
                                "node_id": None, "attempts": 0, "execution_time": None}
        return rid

    def mark_time(self, rid: int, idx: int) -> None:
        """Control-plane timing mark: 1 = picked by the dispatcher, 2 = the worker answered."""
        t = self._tmarks.get(rid)
        if t is not None and not t[idx]:
            t[idx] = time.perf_counter()

    def answered(self, rid: int) -> None:
        """The status API delivered the final row: fold the request's marks into cp_timing
        (queue = submit -> dispatch, worker = dispatch -> worker answer incl. the HTTP hop,
        answer = worker answer -> final status delivered to the client)."""
        t = self._tmarks.pop(rid, None)
        if t is None or not (t[1] and t[2]):
            return
        now = time.perf_counter()
        c = self.cp_timing
        c["answered"] += 1
        c["queue_s"] += t[1] - t[0]
        c["worker_s"] += t[2] - t[1]
        c["answer_s"] += now - t[2]

    def request_fields(self, rid: int):
        """(model_name, prompt) of a request: immutable, so served from this process's own
        rows when it created the request."""
        r = self._live_rows.get(rid) or self._final_rows.get(rid)
        if r is None:
            r = self.get_request(rid)
        return r["model_name"], r["prompt"]

    def get_request(self, rid: int) -> Dict[str, Any]:
        r = self._final_rows.get(rid)
        if r is not None:
            return dict(r)
        rows = self._query("SELECT * FROM inference_request WHERE id=?", (rid,))
        if not rows:
            raise NotFound(f"No InferenceRequest matches the given query (id={rid}).")
        if rows[0]["status"] in ("completed", "failed"):
            self._remember_final(rows[0])
        return rows[0]

    def _remember_final(self, row: Dict[str, Any]) -> None:
        if len(self._final_rows) > 200_000:           # bounded: drop the oldest half
            for k in sorted(self._final_rows)[:100_000]:
                self._final_rows.pop(k, None)
        self._final_rows[int(row["id"])] = dict(row)

    def mark_processing(self, rid: int, node_id: Optional[int] = None):
        t = now_iso()
        self._exec("UPDATE inference_request SET status='processing', started_at=?, node_id=?, "
                   "attempts=attempts+1 WHERE id=?", (t, node_id, rid))
        r = self._live_rows.get(rid)
        if r is not None:
            r.update(status="processing", started_at=t, node_id=node_id,
                     attempts=r["attempts"] + 1)

    def _finish(self, rid: int, sets: str, args: tuple):
        """One terminal UPDATE; the final row comes back by RETURNING (SQLite >= 3.35) in the
        same statement instead of a second SELECT."""
        def tx(c):
            if self._returning:
                return [dict(x) for x in c.execute(
                    f"UPDATE inference_request SET {sets} WHERE id=? RETURNING *",
                    (*args, rid)).fetchall()]
            self._exec(f"UPDATE inference_request SET {sets} WHERE id=?", (*args, rid))
            return self._query("SELECT * FROM inference_request WHERE id=?", (rid,))
        rows = self._call(tx)
        self._live_rows.pop(rid, None)
        if rows:
            self._remember_final(rows[0])
        self._notify_final(rid)
        if self.on_final is not None:
            self.on_final(rid)

    def mark_completed(self, rid: int, result: str, execution_time: Optional[float] = None):
        self._finish(rid, "status='completed', result=?, completed_at=?, execution_time=?",
                     (result, now_iso(), execution_time))

    def mark_failed(self, rid: int, error: str):
        self._finish(rid, "status='failed', error=?, completed_at=?", (error, now_iso()))

    def _notify_final(self, rid: int):
        with self._wlock:
            ev = self._waiters.get(rid)
            aws = self._awaiters.pop(rid, None)
        if ev is not None:
            ev.set()
        if not aws:
            return
        import asyncio
        try:
            here = asyncio.get_running_loop()
        except RuntimeError:
            here = None
        for loop, fut in aws:
            if loop is here:                   # the waiter's own loop: no cross-thread wake-up
                fut.done() or fut.set_result(True)
            else:
                loop.call_soon_threadsafe(lambda f=fut: f.done() or f.set_result(True))

    async def wait_final_async(self, rid: int, timeout_s: float) -> Dict[str, Any]:
        """``wait_final`` for asyncio servers: no thread is held while waiting."""
        import asyncio
        loop = asyncio.get_running_loop()
        fut = loop.create_future()
        with self._wlock:
            self._awaiters.setdefault(rid, []).append((loop, fut))
        deadline = loop.time() + max(0.0, timeout_s)
        first = True
        try:
            while True:
                r = self._final_rows.get(rid)
                live = self._live_rows.get(rid) if first else None
                first = False
                if r is None and live is not None:
                    r = dict(live)                # created here, not finished: no SELECT
                elif r is None:
                    r = await asyncio.wrap_future(self.submit(
                        lambda c: [dict(x) for x in c.execute(
                            "SELECT * FROM inference_request WHERE id=?", (rid,)).fetchall()]))
                    if not r:
                        raise NotFound(f"No InferenceRequest matches the given query (id={rid}).")
                    r = r[0]
                else:
                    r = dict(r)
                left = deadline - loop.time()
                if r["status"] in ("completed", "failed") or left <= 0:
                    return r
                try:
                    await asyncio.wait_for(asyncio.shield(fut), min(left, 2.0))
                except asyncio.TimeoutError:
                    pass
        finally:
            with self._wlock:
                lst = self._awaiters.get(rid)
                if lst is not None:
                    lst[:] = [x for x in lst if x[1] is not fut]
                    if not lst:
                        self._awaiters.pop(rid, None)

    def wait_final(self, rid: int, timeout_s: float) -> Dict[str, Any]:
        """The request's row once it is completed / failed, or as it stands after
        ``timeout_s`` (long-poll support for the status API). Each waiter sleeps on its own
        request's event, set by this process's dispatcher (no thundering herd); a row
        finished by another process is seen within 2 s."""
        import time as _t
        deadline = _t.monotonic() + max(0.0, timeout_s)
        with self._wlock:
            ev = self._waiters.setdefault(rid, threading.Event())
        try:
            while True:
                r = self.get_request(rid)       # served from the terminal-row cache once set
                left = deadline - _t.monotonic()
                if r["status"] in ("completed", "failed") or left <= 0:
                    return r
                ev.wait(min(left, 2.0))
        finally:
            with self._wlock:
                if self._waiters.get(rid) is ev:
                    del self._waiters[rid]

    def requeue(self, rid: int):
        self._final_rows.pop(rid, None)
        r = self._live_rows.get(rid)
        if r is not None:
            r.update(status="pending", node_id=None)
        self._exec("UPDATE inference_request SET status='pending', node_id=NULL WHERE id=?", (rid,))

    def recent_requests(self, n: int = 10) -> List[Dict[str, Any]]:
        return self._query("SELECT * FROM inference_request ORDER BY created_at DESC, id DESC "
                           "LIMIT ?", (n,))

    def count_requests(self, status: Optional[str] = None) -> int:
        if status is None:
            return int(self._query("SELECT COUNT(*) AS n FROM inference_request")[0]["n"])
        return int(self._query("SELECT COUNT(*) AS n FROM inference_request WHERE status=?",
                               (status,))[0]["n"])

    def pending_ids(self) -> List[int]:
        return [r["id"] for r in self._query("SELECT id FROM inference_request WHERE "
                                             "status='pending' ORDER BY id")]

    def recover(self, policy: str = "requeue") -> List[int]:
        """Requests left in 'processing' by a crash/restart: re-queue (default) or fail."""
        stale = [r["id"] for r in self._query("SELECT id FROM inference_request WHERE "
                                              "status='processing'")]
        for rid in stale:
            if policy == "fail":
                self.mark_failed(rid, "Fatal error: master restarted while processing")
            else:
                self.requeue(rid)
        return stale
