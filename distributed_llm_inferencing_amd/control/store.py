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
after ``migrate``; here the schema is created on startup. One connection per thread with a
process-wide write lock (the reference mutated sqlite from unbounded threads, §5.2).
Extensions: node ``resources``/``gpu_id``/``role`` columns, request timing + node columns,
and ``recover()`` which re-queues requests orphaned in ``processing`` by a restart (§5.4).
"""
from __future__ import annotations

import json
import sqlite3
import threading
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


class Store:
    def __init__(self, path: str = ":memory:"):
        self.path = path
        self._lock = threading.RLock()
        self._final = threading.Condition()      # signalled when a request completes / fails
        self._local = threading.local()
        self._shared = None
        if path == ":memory:":
            # one shared connection (an in-memory db is per-connection)
            self._shared = sqlite3.connect(":memory:", check_same_thread=False)
            self._shared.row_factory = sqlite3.Row
            self._shared.execute("PRAGMA foreign_keys = ON")
        with self._lock:
            self._conn().executescript(_SCHEMA)
            self._conn().commit()

    def _conn(self) -> sqlite3.Connection:
        if self._shared is not None:
            return self._shared
        c = getattr(self._local, "conn", None)
        if c is None:
            c = sqlite3.connect(self.path, timeout=30, check_same_thread=False)
            c.row_factory = sqlite3.Row
            c.execute("PRAGMA foreign_keys = ON")
            c.execute("PRAGMA journal_mode = WAL")
            self._local.conn = c
        return c

    def _exec(self, sql: str, args=()):
        with self._lock:
            c = self._conn()
            cur = c.execute(sql, args)
            c.commit()
            return cur

    def _query(self, sql: str, args=()) -> List[Dict[str, Any]]:
        with self._lock:
            return [dict(r) for r in self._conn().execute(sql, args).fetchall()]

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
        with self._lock:
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
        cur = self._exec("INSERT INTO inference_request (model_name, prompt, status, created_at)"
                         " VALUES (?,?, 'pending', ?)", (model_name, prompt, now_iso()))
        return int(cur.lastrowid)

    def get_request(self, rid: int) -> Dict[str, Any]:
        rows = self._query("SELECT * FROM inference_request WHERE id=?", (rid,))
        if not rows:
            raise NotFound(f"No InferenceRequest matches the given query (id={rid}).")
        return rows[0]

    def mark_processing(self, rid: int, node_id: Optional[int] = None):
        self._exec("UPDATE inference_request SET status='processing', started_at=?, node_id=?, "
                   "attempts=attempts+1 WHERE id=?", (now_iso(), node_id, rid))

    def mark_completed(self, rid: int, result: str, execution_time: Optional[float] = None):
        self._exec("UPDATE inference_request SET status='completed', result=?, completed_at=?, "
                   "execution_time=? WHERE id=?", (result, now_iso(), execution_time, rid))
        self._notify_final()

    def mark_failed(self, rid: int, error: str):
        self._exec("UPDATE inference_request SET status='failed', error=?, completed_at=? "
                   "WHERE id=?", (error, now_iso(), rid))
        self._notify_final()

    def _notify_final(self):
        with self._final:
            self._final.notify_all()

    def wait_final(self, rid: int, timeout_s: float) -> Dict[str, Any]:
        """The request's row once it is completed / failed, or as it stands after
        ``timeout_s`` (long-poll support for the status API). Woken by this process's
        dispatcher; rows finished by another process are seen within 0.1 s."""
        import time as _t
        deadline = _t.monotonic() + max(0.0, timeout_s)
        while True:
            r = self.get_request(rid)
            left = deadline - _t.monotonic()
            if r["status"] in ("completed", "failed") or left <= 0:
                return r
            with self._final:
                self._final.wait(min(left, 0.1))

    def requeue(self, rid: int):
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
