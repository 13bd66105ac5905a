"""Failure detector / heartbeat monitor.

Reference: health is probed only when the UI polls ``/api/nodes/status/``; one
``RequestException`` marks a node inactive FOREVER (inactive nodes are never re-probed,
``views.py:88-105``). Here a background thread probes every node (active or not) every
``interval`` seconds:

* success -> is_active = True (automatic re-activation), last_heartbeat = now, the node's
  resources cached, and its reported ``loaded_shards`` synced into the model_shard table
  (in the reference nothing ever created those rows except the Django admin);
* ``fail_threshold`` consecutive failures -> is_active = False;
* the dispatcher can report connection errors (``report_failure``) for faster detection.
"""
from __future__ import annotations

import logging
import threading
from typing import Optional

import requests

from .store import now_iso

log = logging.getLogger("dli.health")
HEALTH_TIMEOUT = 5          # views.py:91,122


def probe(url: str, headers: Optional[dict] = None, timeout: float = HEALTH_TIMEOUT,
          session=None) -> dict:
    http = session or requests
    r = http.get(f"{url}/health", timeout=timeout, headers=headers or {})
    if r.status_code != 200:
        raise requests.RequestException(f"status {r.status_code}: {r.text[:200]}")
    return r.json()


class HealthMonitor:
    def __init__(self, store, settings, interval: float = 10.0, fail_threshold: int = 2,
                 session=None):
        self.store, self.settings = store, settings
        self.interval = interval
        self.fail_threshold = fail_threshold
        self.http = session or requests.Session()
        self._stop = threading.Event()
        self._t: Optional[threading.Thread] = None
        self.rounds = 0

    def headers(self) -> dict:
        return ({"Authorization": f"Bearer {self.settings.auth_key}"}
                if self.settings.auth_key else {})

    def start(self):
        self._t = threading.Thread(target=self._run, name="dli-health", daemon=True)
        self._t.start()

    def stop(self):
        self._stop.set()
        if self._t:
            self._t.join(5)

    def _run(self):
        while not self._stop.wait(self.interval):
            self.check_all()

    def check_all(self):
        for node in self.store.list_nodes():
            self.check(node)
        self.rounds += 1

    def check(self, node: dict) -> Optional[dict]:
        try:
            data = probe(node["url"], self.headers(), session=self.http)
        except Exception as e:  # noqa: BLE001
            self.report_failure(node["id"], str(e))
            return None
        self.store.update_node(node["id"], is_active=True, last_heartbeat=now_iso(),
                               resources=data.get("resources"), failures=0)
        self.sync_shards(node["id"], data.get("loaded_shards") or [])
        return data

    def sync_shards(self, node_id: int, loaded: list):
        for s in loaded:
            try:
                self.store.add_shard(node_id, s["model_name"], int(s["shard_id"]), True,
                                     s.get("path"))
            except Exception as e:  # noqa: BLE001
                log.warning("shard sync failed for node %s: %s", node_id, e)

    def report_failure(self, node_id: int, err: str):
        try:
            node = self.store.get_node(node_id)
        except KeyError:
            return
        fails = int(node.get("failures") or 0) + 1
        fields = {"failures": fails}
        if fails >= self.fail_threshold and node["is_active"]:
            fields["is_active"] = False
            log.warning("node %s (%s) marked inactive: %s", node_id, node["hostname"], err)
        self.store.update_node(node_id, **fields)
