"""Master HTTP service: API-compatible replacement of the reference's Django master.

Routes, form fields, JSON shapes, status codes and messages follow
``master/dashboard/urls.py:6-16`` and ``views.py``:

    GET  /                              dashboard page (counts + 5 recent)
    GET  /nodes/                        node management page
    GET  /inference/                    inference page (10 recent)
    GET  /api/nodes/status/             {"nodes": [...]} live /health probe of active nodes
    POST /api/nodes/add/                form: hostname, ip_address, port
    POST /api/nodes/remove/<id>/        unload shards on the node, delete it
    POST /api/inference/submit/         form: model_name, prompt -> {"request_id"}
    GET  /api/inference/status/<id>/    request state machine view
    GET  /api/inference/recent/         10 newest requests
    /admin/                             table browser (Django admin stand-in, admin.py:4-19)

Additions: POST /api/shards/register/ (the only way the reference could create ModelShard
rows was the Django admin), POST /api/shards/delete/<id>/, GET /api/shards/,
GET /metrics (queue depth, request counts, dispatcher stats), GET /healthz.
Submissions go to a request queue drained by the dispatcher (one asyncio loop for every
in-flight worker call; no thread per request); a background heartbeat monitor keeps node
state fresh. GET /api/inference/status/<id>/?wait=<s> long-polls until completion.
"""
from __future__ import annotations

import logging
import os
import time
from pathlib import Path
from typing import Optional

import requests
from flask import Flask, jsonify, render_template, request, session

from ..config import Settings, get_settings
from .dispatcher import make_dispatcher
from .health import HealthMonitor, probe
from .queue import make_queue
from .store import NotFound, Store, now_iso

log = logging.getLogger("dli.master")
TEMPLATES = Path(__file__).resolve().parent / "templates"


class MasterState:
    def __init__(self, settings: Settings, store: Store, start_background: bool = True,
                 dispatch_workers: Optional[int] = None, health_interval: float = 10.0):
        self.settings = settings
        self.store = store
        # serve-master --procs N: this process's rank; peers share the database and hear of
        # each other's finished requests (control/peers.py)
        self.rank = int(os.environ.get("DLI_MASTER_RANK", "0"))
        self.nprocs = int(os.environ.get("DLI_MASTER_PROCS", "1"))
        self.notifier = None
        if self.nprocs > 1:
            from .peers import PeerNotifier
            self.notifier = PeerNotifier(self.rank, self.nprocs,
                                         int(os.environ.get("DLI_MASTER_NOTIFY_PORT", "47600")))
            store.on_final = self.notifier.publish
        self.queue = make_queue(settings.queue_backend, store, settings)
        self.health = HealthMonitor(store, settings, interval=health_interval)
        self.dispatcher = make_dispatcher(store, self.queue, settings,
                                          num_workers=dispatch_workers or
                                          settings.dispatch_workers,
                                          on_node_error=self.health.report_failure)
        if self.rank == 0:
            recovered = store.recover("requeue")
            for rid in store.pending_ids():
                self.queue.put(rid)
            if recovered:
                log.warning("re-queued %d requests orphaned in 'processing'", len(recovered))
        if start_background:
            # an ASGI front (serve-master --server uvicorn / aiohttp) runs the async
            # dispatcher on its own event loop (control/asgi.py starts it there)
            if not (os.environ.get("DLI_DISPATCH_ON_SERVER_LOOP", "0") == "1"
                    and hasattr(self.dispatcher, "start_on_loop")):
                self.dispatcher.start()
            if self.rank == 0:
                self.health.start()

    def shutdown(self):
        self.dispatcher.stop()
        self.health.stop()


# ----------------------------------------------------------------------------- validation
def _required_str(form, name, max_len=None):
    v = form.get(name)
    if v is None or str(v).strip() == "":
        return None, ["This field is required."]
    v = str(v)
    if max_len and len(v) > max_len:
        return None, [f"Ensure this value has at most {max_len} characters (it has {len(v)})."]
    return v, None


def validate_node_form(form):
    errors, data = {}, {}
    for f in ("hostname", "ip_address"):
        v, e = _required_str(form, f, 255)
        if e:
            errors[f] = e
        data[f] = v
    p = form.get("port")
    if p is None or str(p).strip() == "":
        errors["port"] = ["This field is required."]
    else:
        try:
            data["port"] = int(str(p).strip())
        except ValueError:
            errors["port"] = ["Enter a whole number."]
    return data, errors


def validate_inference_form(form):
    errors, data = {}, {}
    v, e = _required_str(form, "model_name", 255)
    if e:
        errors["model_name"] = e
    data["model_name"] = v
    v, e = _required_str(form, "prompt")
    if e:
        errors["prompt"] = e
    data["prompt"] = v
    return data, errors


def _flash(msg: str, kind: str):
    session["status_message"] = msg
    session["status_type"] = kind


def _pop_flash():
    return session.pop("status_message", None), session.pop("status_type", "info")


# ----------------------------------------------------------------------------- app
def create_master_app(settings: Optional[Settings] = None, store: Optional[Store] = None,
                      start_background: bool = True, **state_kw) -> Flask:
    settings = settings or get_settings()
    store = store or Store(settings.master_db)
    app = Flask(__name__, template_folder=str(TEMPLATES))
    app.secret_key = settings.secret_key
    app.config["DEBUG"] = settings.debug
    st = MasterState(settings, store, start_background=start_background, **state_kw)
    app.extensions["dli"] = st
    http = requests.Session()

    def auth_headers():
        return ({"Authorization": f"Bearer {settings.auth_key}"} if settings.auth_key else {})

    # -------------------------------------------------------------- pages
    @app.get("/")
    def dashboard():
        ctx = dict(active_nodes=store.count_nodes(True), total_nodes=store.count_nodes(),
                   pending_requests=store.count_requests("pending"),
                   processing_requests=store.count_requests("processing"),
                   completed_requests=store.count_requests("completed"),
                   failed_requests=store.count_requests("failed"),
                   recent_requests=store.recent_requests(5), page="dashboard")
        return render_template("dashboard.html", **ctx)

    @app.get("/nodes/")
    def node_management():
        msg, kind = _pop_flash()
        return render_template("node_management.html", nodes=store.list_nodes(),
                               status_message=msg, status_type=kind, page="nodes")

    @app.get("/inference/")
    def inference_page():
        msg, kind = _pop_flash()
        return render_template("inference.html", recent_requests=store.recent_requests(10),
                               status_message=msg, status_type=kind, page="inference")

    # -------------------------------------------------------------- node API
    @app.get("/api/nodes/status/")
    def node_status():
        nodes = []
        for node in store.list_nodes():
            d = {"id": node["id"], "hostname": node["hostname"],
                 "ip_address": node["ip_address"], "port": node["port"],
                 "is_active": node["is_active"], "last_heartbeat": node["last_heartbeat"]}
            if node["is_active"]:
                try:
                    health = probe(node["url"], auth_headers(), session=http)
                    d["resources"] = health.get("resources", {})
                    d["loaded_shards"] = health.get("loaded_shards", [])
                    hb = now_iso()
                    store.update_node(node["id"], last_heartbeat=hb,
                                      resources=d["resources"], failures=0)
                    st.health.sync_shards(node["id"], d["loaded_shards"])
                except requests.RequestException as e:
                    d["error"] = f"Connection error: {e}"
                    log.warning("Health check failed for node %s: %s", node["hostname"], e)
                    store.update_node(node["id"], is_active=False)
                    d["is_active"] = False
            nodes.append(d)
        return jsonify({"nodes": nodes})

    @app.post("/api/nodes/add/")
    def add_node():
        data, errors = validate_node_form(request.form)
        if errors:
            return jsonify({"status": "error",
                            "message": "Form validation failed. Please correct the errors and "
                                       "try again.", "errors": errors}), 400
        url = f"http://{data['ip_address']}:{data['port']}"
        try:
            r = http.get(f"{url}/health", timeout=5, headers=auth_headers())
            if r.status_code != 200:
                return jsonify({"status": "error",
                                "message": f"Node returned status code {r.status_code}. "
                                           f"Response: {r.text}"}), 400
            health = r.json()
        except requests.RequestException as e:
            return jsonify({"status": "error",
                            "message": f"Could not connect to node: {e}. Please check the "
                                       "hostname, IP, and port."}), 400
        except Exception as e:  # noqa: BLE001
            return jsonify({"status": "error",
                            "message": f"An unexpected error occurred: {e}"}), 500
        nid = store.add_node(data["hostname"], data["ip_address"], data["port"], True, now_iso())
        store.update_node(nid, resources=health.get("resources"))
        st.health.sync_shards(nid, health.get("loaded_shards") or [])
        _flash(f"Node {data['hostname']} ({data['ip_address']}) added successfully", "success")
        return jsonify({"status": "success", "node_id": nid, "hostname": data["hostname"],
                        "message": f"Node {data['hostname']} added successfully"})

    @app.post("/api/nodes/remove/<int:node_id>/")
    def remove_node(node_id):
        try:
            node = store.get_node(node_id)
            errs = []
            for sh in store.shards(node_id=node_id):
                try:
                    r = http.post(f"{node['url']}/unload_model",
                                  json={"model_name": sh["model_name"]}, timeout=10,
                                  headers=auth_headers())
                    if r.status_code != 200:
                        errs.append(f"Failed to unload shard {sh['shard_id']} of model "
                                    f"{sh['model_name']}: {r.text}")
                except requests.RequestException as e:
                    errs.append(f"Connection error while unloading shard {sh['shard_id']}: {e}")
            store.delete_node(node_id)
            if errs:
                msg = f"Node {node['hostname']} removed, but with warnings: {'; '.join(errs)}"
                _flash(msg, "warning")
            else:
                msg = f"Node {node['hostname']} removed successfully"
                _flash(msg, "success")
            return jsonify({"status": "success", "message": msg, "warnings": errs or None})
        except Exception as e:  # noqa: BLE001 (unknown id -> 500, as views.py:212)
            msg = f"Failed to remove node: {e.args[0] if isinstance(e, NotFound) else e}"
            _flash(msg, "error")
            return jsonify({"status": "error", "message": msg}), 500

    # -------------------------------------------------------------- inference API
    @app.post("/api/inference/submit/")
    def submit_inference():
        data, errors = validate_inference_form(request.form)
        if errors:
            return jsonify({"status": "error",
                            "message": "Form validation failed. Please correct the errors and "
                                       "try again.", "errors": errors}), 400
        rid = store.create_request(data["model_name"], data["prompt"])
        st.dispatcher.submit(rid)
        _flash("Inference request submitted successfully", "success")
        return jsonify({"status": "success", "message": "Inference request submitted "
                        "successfully", "request_id": rid})

    @app.get("/api/inference/status/<int:request_id>/")
    def inference_status(request_id):
        try:
            # optional long poll (?wait=<s>, <= 60): answer when the request completes or
            # fails, or after the wait — one call per request instead of a polling storm;
            # without it the route answers at once, as the reference's does
            wait = min(float(request.args.get("wait", 0) or 0), 60.0)
            r = store.wait_final(request_id, wait) if wait > 0 else store.get_request(request_id)
            return jsonify({"id": r["id"], "status": r["status"], "model_name": r["model_name"],
                            "prompt": r["prompt"], "result": r["result"], "error": r["error"],
                            "created_at": r["created_at"], "completed_at": r["completed_at"]})
        except Exception as e:  # noqa: BLE001
            m = e.args[0] if isinstance(e, NotFound) else str(e)
            return jsonify({"status": "error",
                            "message": f"Error retrieving inference status: {m}"}), 500

    @app.get("/api/inference/recent/")
    def recent_inferences():
        try:
            return jsonify({"requests": [
                {"id": r["id"], "model_name": r["model_name"], "status": r["status"],
                 "created_at": r["created_at"], "completed_at": r["completed_at"]}
                for r in store.recent_requests(10)]})
        except Exception as e:  # noqa: BLE001
            return jsonify({"status": "error",
                            "message": f"Error retrieving recent inferences: {e}"}), 500

    # -------------------------------------------------------------- shards / admin / metrics
    @app.get("/api/shards/")
    def list_shards():
        return jsonify({"shards": store.shards(model_name=request.args.get("model_name"))})

    @app.post("/api/shards/register/")
    def register_shard():
        f = request.form if request.form else (request.get_json(silent=True) or {})
        try:
            node_id, shard_id = int(f["node_id"]), int(f["shard_id"])
            model = str(f["model_name"])
        except (KeyError, ValueError, TypeError):
            return jsonify({"status": "error",
                            "message": "node_id, model_name and shard_id are required"}), 400
        try:
            store.get_node(node_id)
        except NotFound as e:
            return jsonify({"status": "error", "message": e.args[0]}), 404
        loaded = str(f.get("is_loaded", "1")).lower() in ("1", "true", "yes", "on")
        pk = store.add_shard(node_id, model, shard_id, loaded, f.get("path"))
        return jsonify({"status": "success", "id": pk})

    @app.post("/api/shards/delete/<int:pk>/")
    def delete_shard(pk):
        store.delete_shard(pk)
        return jsonify({"status": "success"})

    @app.get("/admin/")
    def admin():
        return render_template("admin.html", nodes=store.list_nodes(), shards=store.shards(),
                               requests=store.recent_requests(50), page="admin")

    @app.get("/metrics")
    def metrics():
        return jsonify({
            "queue_backend": st.queue.name, "queue_depth": st.queue.qsize(),
            "requests": {s: store.count_requests(s) for s in
                         ("pending", "processing", "completed", "failed")},
            "nodes": {"total": store.count_nodes(), "active": store.count_nodes(True)},
            "dispatcher": {"workers": st.dispatcher.num_workers,
                           "processed": st.dispatcher.processed,
                           "inflight": dict(st.dispatcher.inflight)},
            "health_rounds": st.health.rounds,
            # mean control-plane latency per request answered by a long poll of this process
            "control_plane_latency_s": {
                k: round(v / max(1, store.cp_timing["answered"]), 4)
                for k, v in store.cp_timing.items() if k != "answered"}
            | {"answered": store.cp_timing["answered"]}})

    @app.get("/healthz")
    def healthz():
        return jsonify({"status": "ok"})

    return app


def main(argv=None):
    import argparse
    ap = argparse.ArgumentParser("dli serve-master")
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--port", type=int, default=8000)
    ap.add_argument("--server", default="werkzeug", choices=["werkzeug", "uvicorn", "aiohttp"],
                    help="werkzeug: threaded WSGI server (a thread per connection); uvicorn: "
                         "ASGI front (control/asgi.py: async submit and status long polls) "
                         "over the same Flask app; aiohttp: the same ASGI front on aiohttp's "
                         "C HTTP parser (utils/aioserve.py)")
    ap.add_argument("--procs", type=int, default=int(os.environ.get("DLI_MASTER_PROCS", "1")),
                    help="aiohttp: N master processes on one port and one database "
                         "(control/peers.py)")
    a = ap.parse_args(argv)
    if a.server in ("aiohttp", "uvicorn"):
        os.environ.setdefault("DLI_DISPATCH_ON_SERVER_LOOP", "1")
    if a.server == "aiohttp":
        if a.procs > 1 and "DLI_MASTER_RANK" not in os.environ:
            return _spawn_procs(a, argv)
        from .asgi import create_asgi_app
        from ..utils.aioserve import run_asgi
        from ..utils.log import setup_logging
        rank = os.environ.get("DLI_MASTER_RANK")
        setup_logging("master" if rank in (None, "0") else f"master{rank}")
        run_asgi(create_asgi_app(create_master_app()), host=a.host, port=a.port,
                 reuse_port=a.procs > 1)
        return
    if a.server == "uvicorn":
        # ASGI front: status long polls as coroutines, the Flask app behind a WSGI adapter
        import uvicorn

        from .asgi import create_asgi_app
        from ..utils.log import setup_logging
        setup_logging("master")
        uvicorn.run(create_asgi_app(create_master_app()), host=a.host, port=a.port,
                    log_level="warning", timeout_keep_alive=75, backlog=4096)
        return
    from ..utils.log import setup_logging
    setup_logging("master")
    # werkzeug's thread-per-request server + the threaded dispatcher: the store's database
    # thread (inline mode is for the event-loop fronts above, whose callers are one loop;
    # with many request threads one RLock on the caller's thread convoys). DLI_STORE_INLINE
    # overrides.
    s = get_settings()
    env_inline = os.environ.get("DLI_STORE_INLINE")
    app = create_master_app(s, store=Store(s.master_db, inline=(
        env_inline == "1" if env_inline is not None else False)))
    app.run(host=a.host, port=a.port, threaded=True)


def _spawn_procs(a, argv) -> int:
    """serve-master --server aiohttp --procs N: N child processes (rank 0..N-1) serving the
    same port (SO_REUSEPORT) and database; exits with the first child's failure."""
    import signal
    import subprocess
    import sys
    settings = get_settings()
    if settings.master_db in ("", ":memory:"):
        raise SystemExit("--procs > 1 needs a database file (MASTER_DB) the processes share")
    procs = []
    for r in range(a.procs):
        env = dict(os.environ, DLI_MASTER_RANK=str(r), DLI_MASTER_PROCS=str(a.procs))
        procs.append(subprocess.Popen([sys.executable, "-m", "distributed_llm_inferencing_amd.cli",
                                       "serve-master", *(argv or [])], env=env))
        if r == 0:
            time.sleep(1.0)             # rank 0 creates the schema and re-queues first

    def stop(*_):
        for p in procs:
            if p.poll() is None:
                p.terminate()
    signal.signal(signal.SIGTERM, stop)
    signal.signal(signal.SIGINT, stop)
    rc = 0
    try:
        while True:
            for p in procs:
                r = p.poll()
                if r is not None:
                    stop()
                    for q in procs:
                        try:
                            q.wait(10)
                        except subprocess.TimeoutExpired:
                            q.kill()
                    return r or rc
            time.sleep(0.5)
    finally:
        stop()


if __name__ == "__main__":
    main()
