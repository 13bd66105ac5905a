"""T1/T2 control-plane tests: sqlite store, queues, master API contract (Appendix A),
worker API contract (Appendix B), and master -> worker dispatch over real HTTP on localhost
with the CPU engine (config 1: gpt2 on a CPU worker)."""
import threading
from pathlib import Path
import time

import pytest
import requests
import torch
from werkzeug.serving import make_server

from distributed_llm_inferencing_amd.config import Settings
from distributed_llm_inferencing_amd.control.master import create_master_app
from distributed_llm_inferencing_amd.control.queue import InProcQueue, SqliteQueue, make_queue
from distributed_llm_inferencing_amd.control.store import NotFound, Store
from distributed_llm_inferencing_amd.worker.server import create_worker_app

SMALL = dict(max_batch=8, max_model_len=128, num_blocks=64)


class Server:
    def __init__(self, app):
        self.srv = make_server("127.0.0.1", 0, app, threaded=True)
        self.port = self.srv.server_port
        self.t = threading.Thread(target=self.srv.serve_forever, daemon=True)
        self.t.start()

    @property
    def url(self):
        return f"http://127.0.0.1:{self.port}"

    def close(self):
        self.srv.shutdown()


def settings(tmp_path, **kw):
    s = Settings()
    s.master_db = str(tmp_path / "db.sqlite3")
    s.model_cache_dir = str(tmp_path / "cache")
    s.dispatch_workers = 8
    for k, v in kw.items():
        setattr(s, k, v)
    return s


# ----------------------------------------------------------------------------- store / queue
def test_store_state_machine(tmp_path):
    st = Store(str(tmp_path / "s.db"))
    n = st.add_node("w1", "127.0.0.1", 5000)
    assert st.get_node(n)["url"] == "http://127.0.0.1:5000"
    st.add_shard(n, "gpt2", 0, True)
    st.add_shard(n, "gpt2", 0, True)                 # unique (model, shard) -> upsert
    assert len(st.shards("gpt2")) == 1
    rid = st.create_request("gpt2", "hi")
    assert st.get_request(rid)["status"] == "pending"
    st.mark_processing(rid, n)
    assert st.recover() == [rid] and st.get_request(rid)["status"] == "pending"
    st.mark_processing(rid, n)
    st.mark_completed(rid, "out", 0.5)
    r = st.get_request(rid)
    assert r["status"] == "completed" and r["result"] == "out" and r["completed_at"]
    st.delete_node(n)                                # cascade removes shards
    assert st.shards() == []
    with pytest.raises(NotFound):
        st.get_node(n)


def test_queues(tmp_path):
    q = InProcQueue()
    q.put(3)
    assert q.get(0.1) == 3 and q.get(0.01) is None
    st = Store(str(tmp_path / "q.db"))
    sq = SqliteQueue(st)
    a, b = st.create_request("m", "p"), st.create_request("m", "p")
    assert sq.get(0.5) == a and sq.get(0.5) == b and sq.get(0.05) is None
    assert make_queue("redis", st, Settings()).name in ("redis", "inproc")


# ----------------------------------------------------------------------------- worker API
@pytest.fixture()
def worker(tmp_path):
    app = create_worker_app(settings(tmp_path), device="cpu", engine_kwargs=SMALL)
    return app.test_client()


def test_worker_health_and_load(worker):
    h = worker.get("/health").get_json()
    assert h["status"] == "healthy"
    assert set(h["resources"]) >= {"cpu", "memory", "gpu", "gpu_available", "device"}
    assert h["resources"]["device"] == "cpu"
    assert worker.post("/load_model", json={}).status_code == 400
    r = worker.post("/load_model", json={"model_name": "gpt2-tiny"}).get_json()
    assert r["status"] == "success" and "loaded successfully on cpu" in r["message"]
    r = worker.post("/load_model", json={"model_name": "gpt2-tiny"}).get_json()
    assert "already loaded" in r["message"]
    assert worker.get("/health").get_json()["loaded_models"] == ["gpt2-tiny"]
    assert worker.post("/load_model", json={"model_name": "nope"}).status_code == 500
    assert worker.post("/unload_model", json={"model_name": "gpt2-tiny"}).status_code == 200
    assert worker.get("/health").get_json()["loaded_models"] == []


def test_worker_inference_contract(worker):
    assert worker.post("/inference", json={"model_name": "gpt2-tiny"}).status_code == 400
    r = worker.post("/inference", json={"model_name": "llama-tiny", "prompt": "Hello",
                                        "max_length": 20})
    d = r.get_json()
    assert r.status_code == 200 and d["status"] == "success"
    assert d["result"].startswith("Hello") and d["execution_time"] > 0
    assert d["output_tokens"] == 20 - 5


def test_worker_concurrent_requests_are_batched(worker):
    worker.post("/load_model", json={"model_name": "llama-tiny"})
    out = [None] * 6

    def call(i):
        out[i] = worker.post("/inference", json={"model_name": "llama-tiny",
                                                 "prompt": f"req {i}", "max_length": 24})
    ts = [threading.Thread(target=call, args=(i,)) for i in range(6)]
    [t.start() for t in ts]
    [t.join() for t in ts]
    assert all(r.status_code == 200 for r in out)
    m = worker.get("/metrics").get_json()["engines"]["llama-tiny"]
    assert m["finished_requests"] == 6
    assert m["decode_steps"] < 6 * 17            # shared decode steps


def test_worker_timeout_408(worker):
    r = worker.post("/inference", json={"model_name": "llama-tiny", "prompt": "x" * 10,
                                        "max_length": 120, "timeout": 0})
    assert r.status_code == 408


def test_worker_auth(tmp_path):
    app = create_worker_app(settings(tmp_path, auth_enabled=True, auth_key="k"), device="cpu",
                            engine_kwargs=SMALL).test_client()
    assert app.get("/health").status_code == 401
    assert app.get("/health", headers={"Authorization": "Bearer k"}).status_code == 200


def test_worker_ssh_setup_contract(worker):
    assert worker.post("/ssh_setup", json={"host": "h"}).status_code == 400
    r = worker.post("/ssh_setup", json={"host": "127.0.0.1", "port": 1, "username": "u",
                                        "password": "p"})
    assert r.status_code == 500 and "SSH connection failed" in r.get_json()["message"]


def test_shard_export_load_and_sharded_inference(tmp_path, worker):
    from distributed_llm_inferencing_amd.shard.writer import export_shards
    paths = export_shards("llama-tiny", 2, str(tmp_path / "shards"), log=lambda *a: None)
    meta = (paths[1] / "metadata.json").read_text()
    assert '"end_layer": 3' in meta and '"total_layers": 4' in meta
    # shard_id 0 accepted (the reference rejected it)
    r = worker.post("/load_shard", json={"model_name": "llama-tiny", "shard_id": 0,
                                         "shard_path": str(paths[0])})
    assert r.status_code == 200, r.get_json()
    # a partial shard set must be refused, not run as a whole model
    r = worker.post("/inference", json={"model_name": "llama-tiny", "prompt": "abc",
                                        "shard_ids": [0]})
    assert r.status_code == 500 and "cannot run a partial model" in r.get_json()["message"]
    worker.post("/load_shard", json={"model_name": "llama-tiny", "shard_id": 1,
                                     "shard_path": str(paths[1])})
    h = worker.get("/health").get_json()
    assert sorted(s["shard_id"] for s in h["loaded_shards"]) == [0, 1]
    body = {"model_name": "llama-tiny", "prompt": "abc", "max_length": 16, "temperature": 0}
    sharded = worker.post("/inference", json={**body, "shard_ids": [0, 1]}).get_json()
    full = worker.post("/inference", json=body).get_json()
    assert sharded["status"] == "success"
    assert sharded["result"] == full["result"]       # same weights: exported == random init


# ----------------------------------------------------------------------------- master API
@pytest.fixture()
def master(tmp_path):
    app = create_master_app(settings(tmp_path), start_background=True, dispatch_workers=2,
                            health_interval=0.5)
    yield app
    app.extensions["dli"].shutdown()


def test_master_pages_and_validation(master):
    c = master.test_client()
    for p in ("/", "/nodes/", "/inference/", "/admin/"):
        assert c.get(p).status_code == 200
    r = c.post("/api/nodes/add/", data={"hostname": "x"})
    assert r.status_code == 400 and set(r.get_json()["errors"]) == {"ip_address", "port"}
    r = c.post("/api/nodes/add/", data={"hostname": "x", "ip_address": "127.0.0.1", "port": 1})
    assert r.status_code == 400 and "Could not connect to node" in r.get_json()["message"]
    r = c.post("/api/inference/submit/", data={"model_name": "gpt2"})
    assert r.status_code == 400 and "prompt" in r.get_json()["errors"]
    assert c.get("/api/inference/status/999/").status_code == 500
    assert c.post("/api/nodes/remove/999/").status_code == 500
    assert c.get("/api/inference/recent/").get_json() == {"requests": []}


def test_end_to_end_dispatch_over_http(tmp_path, master):
    """submit -> queue -> dispatcher -> worker /load_model + /inference -> completed."""
    w = Server(create_worker_app(settings(tmp_path), device="cpu", engine_kwargs=SMALL))
    try:
        c = master.test_client()
        r = c.post("/api/nodes/add/", data={"hostname": "cpu0", "ip_address": "127.0.0.1",
                                            "port": w.port}).get_json()
        assert r["status"] == "success"
        nodes = c.get("/api/nodes/status/").get_json()["nodes"]
        assert nodes[0]["is_active"] and nodes[0]["resources"]["device"] == "cpu"
        rid = c.post("/api/inference/submit/", data={"model_name": "gpt2-tiny",
                                                     "prompt": "Hello"}).get_json()["request_id"]
        deadline = time.time() + 120      # model load + generation; slow under a loaded CPU
        while time.time() < deadline:
            st = c.get(f"/api/inference/status/{rid}/").get_json()
            if st["status"] in ("completed", "failed"):
                break
            time.sleep(0.1)
        assert st["status"] == "completed", st
        assert st["result"].startswith("Hello") and st["completed_at"]
        recent = c.get("/api/inference/recent/").get_json()["requests"]
        assert recent[0]["id"] == rid
        # further requests to the same node skip the /load_model round trip
        rids = [c.post("/api/inference/submit/", data={"model_name": "gpt2-tiny",
                                                       "prompt": f"Hi {i}"}).get_json()[
            "request_id"] for i in range(3)]
        deadline = time.time() + 120
        while time.time() < deadline and any(
                c.get(f"/api/inference/status/{r}/").get_json()["status"] not in
                ("completed", "failed") for r in rids):
            time.sleep(0.1)
        assert all(c.get(f"/api/inference/status/{r}/").get_json()["status"] == "completed"
                   for r in rids)
        assert master.extensions["dli"].dispatcher.load_calls == 1
        m = c.get("/metrics").get_json()
        assert m["requests"]["completed"] == 4
    finally:
        w.close()


def test_master_module_level_wsgi_app(tmp_path, monkeypatch):
    """control/wsgi.py exposes ``application`` (reference master/master/wsgi.py) built from
    the environment; it serves the reference routes."""
    import importlib
    import sys
    monkeypatch.setenv("MASTER_DB", str(tmp_path / "w.sqlite3"))
    monkeypatch.setenv("MODEL_CACHE_DIR", str(tmp_path / "cache"))
    monkeypatch.setenv("DLI_LOG_DIR", str(tmp_path / "logs"))
    sys.modules.pop("distributed_llm_inferencing_amd.control.wsgi", None)
    mod = importlib.import_module("distributed_llm_inferencing_amd.control.wsgi")
    try:
        c = mod.application.test_client()
        assert c.get("/").status_code == 200
        assert c.get("/api/nodes/status/").get_json() == {"nodes": []}
        r = c.post("/api/inference/submit/", data={"model_name": "gpt2", "prompt": "x"})
        assert r.get_json()["status"] == "success"
    finally:
        mod.application.extensions["dli"].shutdown()
        sys.modules.pop("distributed_llm_inferencing_amd.control.wsgi", None)


def test_failover_and_no_nodes(tmp_path, master):
    c = master.test_client()
    rid = c.post("/api/inference/submit/", data={"model_name": "gpt2-tiny",
                                                 "prompt": "x"}).get_json()["request_id"]
    deadline = time.time() + 30
    while time.time() < deadline:
        st = c.get(f"/api/inference/status/{rid}/").get_json()
        if st["status"] == "failed":
            break
        time.sleep(0.05)
    assert st["error"] == "No active worker nodes available"
    # a dead node plus a live one: the request must land on the live one
    w = Server(create_worker_app(settings(tmp_path), device="cpu", engine_kwargs=SMALL))
    try:
        store = master.extensions["dli"].store
        dead = store.add_node("dead", "127.0.0.1", 1, True)
        c.post("/api/nodes/add/", data={"hostname": "live", "ip_address": "127.0.0.1",
                                        "port": w.port})
        rids = [c.post("/api/inference/submit/", data={"model_name": "gpt2-tiny",
                                                       "prompt": f"p{i}"}).get_json()["request_id"]
                for i in range(3)]
        for rid in rids:
            deadline = time.time() + 180        # generous: CPU-loaded parallel test runs
            while time.time() < deadline:
                st = c.get(f"/api/inference/status/{rid}/").get_json()
                if st["status"] in ("completed", "failed"):
                    break
                time.sleep(0.1)
            assert st["status"] == "completed", st
        # the health monitor eventually marks the dead node inactive
        for _ in range(50):
            if not store.get_node(dead)["is_active"]:
                break
            time.sleep(0.1)
        assert not store.get_node(dead)["is_active"]
    finally:
        w.close()


def test_remove_node_unloads(tmp_path, master):
    w = Server(create_worker_app(settings(tmp_path), device="cpu", engine_kwargs=SMALL))
    try:
        c = master.test_client()
        nid = c.post("/api/nodes/add/", data={"hostname": "w", "ip_address": "127.0.0.1",
                                              "port": w.port}).get_json()["node_id"]
        requests.post(f"{w.url}/load_model", json={"model_name": "gpt2-tiny"}, timeout=60)
        c.post("/api/shards/register/", data={"node_id": nid, "model_name": "gpt2-tiny",
                                              "shard_id": 0})
        r = c.post(f"/api/nodes/remove/{nid}/").get_json()
        assert r["status"] == "success" and r["warnings"] is None
        assert requests.get(f"{w.url}/health", timeout=10).json()["loaded_models"] == []
    finally:
        w.close()


def test_dp_replica_plan_and_pipeline_head_routing(tmp_path):
    """serve-cluster: K pipelines of gpus/K ranks; a replica head serves its model as a plain
    node (load_model = already loaded; /inference with or without shard_ids -> pipeline)."""
    from distributed_llm_inferencing_amd.cli import cluster_plan
    from distributed_llm_inferencing_amd.engine.sequence import RequestOutput
    from distributed_llm_inferencing_amd.worker.server import WorkerState
    assert cluster_plan(8, 2) == [(0, "0,1,2,3", 5000, 29600), (1, "4,5,6,7", 5001, 29601)]
    assert [p[1] for p in cluster_plan(8, 8)] == [str(i) for i in range(8)]
    with pytest.raises(ValueError):
        cluster_plan(8, 3)

    class FakePipe:
        calls = 0

        def generate(self, prompt, params=None, timeout=None):
            FakePipe.calls += 1
            return RequestOutput(request_id="x", prompt_ids=[1], output_ids=[2, 3],
                                 finish_reason="length", latency_s=0.1, ttft_s=None,
                                 text=f"{prompt}!")

        def stats(self):
            return {}

    s = settings(tmp_path)
    st = WorkerState(s, "cpu")
    st.pipeline_model, st.pipeline_service, st.pipeline_shards = "llama3-8b", FakePipe(), []
    c = create_worker_app(s, state=st).test_client()
    r = c.post("/load_model", json={"model_name": "llama3-8b"})
    assert r.status_code == 200 and "already loaded" in r.get_json()["message"]
    for extra in ({}, {"shard_ids": [0, 1]}):
        r = c.post("/inference", json={"model_name": "llama3-8b", "prompt": "hi", **extra})
        assert r.status_code == 200 and r.get_json()["result"] == "hi!"
    assert FakePipe.calls == 2 and "llama3-8b" not in st.services


def test_loadgen_end_to_end(tmp_path, master):
    """Load generator through the public master API: concurrent clients, every request
    completes; the worker batches them (continuous batching across HTTP requests)."""
    from distributed_llm_inferencing_amd.loadgen import LoadGen
    # all 6 clients' requests in flight at once (one dispatcher slot each), so the worker
    # batches them into shared steps; polling every 0.1 s (the reference UI polls every 2 s)
    # keeps the pollers from competing with the engine thread for the GIL on a loaded host.
    # Root cause of the earlier flake: 2 dispatcher slots serialised the 12 requests into 6
    # rounds of a 2-row batch, which took > 120 s under CPU contention.
    # one intra-op thread: under pytest-xdist the OpenMP pools of several workers oversubscribe
    # the host's CPUs and spin-wait into one another (every request hit its 60 s deadline)
    threads = torch.get_num_threads()
    torch.set_num_threads(1)
    master.extensions["dli"].shutdown()
    master = create_master_app(settings(tmp_path, master_db=str(tmp_path / "lg.sqlite3")),
                               start_background=True, dispatch_workers=6, health_interval=0.5)
    w = Server(create_worker_app(settings(tmp_path), device="cpu", engine_kwargs=SMALL))
    ms = Server(master)
    try:
        requests.post(f"{ms.url}/api/nodes/add/", data={"hostname": "cpu0",
                                                       "ip_address": "127.0.0.1",
                                                       "port": w.port}, timeout=10)
        lg = LoadGen(ms.url, "gpt2-tiny", poll_s=0.1, timeout_s=240)
        wall = lg.closed_loop([f"hello {i}" for i in range(12)], concurrency=6)
        rep = lg.report(wall)
        assert rep["completed"] == 12 and rep["failed"] == 0, (rep, [
            master.extensions["dli"].store.get_request(r["id"]) for r in lg.results
            if r["status"] != "completed"][:3])
        assert rep["p50_latency_s"] <= rep["p99_latency_s"]
        assert rep["requests_per_s"] > 0
    finally:
        torch.set_num_threads(threads)
        ms.close()
        w.close()
        master.extensions["dli"].shutdown()


def test_worker_health_reports_failed_pipeline(worker):
    """A pipeline head whose ring broke (PipelineService.error set) answers /health with 503,
    so the master's heartbeat takes the node out of rotation."""
    assert worker.get("/health").status_code == 200

    class _Broken:
        error = RuntimeError("stage 3 died")
    worker.application.extensions["dli_worker"].pipeline_service = _Broken()
    r = worker.get("/health")
    assert r.status_code == 503 and "stage 3 died" in r.get_json()["message"]


def test_worker_asgi_front_matches_flask_route(tmp_path):
    """serve-worker --server uvicorn: /inference as a coroutine gives the Flask route's
    JSON / status codes (success, 400, 401, 408), other routes fall through to Flask."""
    import asyncio
    import httpx
    from distributed_llm_inferencing_amd.worker.asgi import create_asgi_app
    flask_app = create_worker_app(settings(tmp_path), device="cpu", engine_kwargs=SMALL)
    flask_app.extensions["dli_worker"].load_model("llama-tiny")
    app = create_asgi_app(flask_app)
    body = {"model_name": "llama-tiny", "prompt": "Hello", "max_length": 20, "temperature": 0}

    async def run():
        tr = httpx.ASGITransport(app=app)
        async with httpx.AsyncClient(transport=tr, base_url="http://w") as c:
            outs = await asyncio.gather(*(c.post("/inference", json=body) for _ in range(4)))
            h = await c.get("/health")
            bad = await c.post("/inference", json={"model_name": "llama-tiny"})
            late = await c.post("/inference", json={**body, "max_length": 120, "timeout": 0})
            return outs, h, bad, late
    outs, h, bad, late = asyncio.run(run())
    want = flask_app.test_client().post("/inference", json=body).get_json()
    for r in outs:
        d = r.json()
        assert r.status_code == 200 and d["result"] == want["result"]
        assert d["output_tokens"] == want["output_tokens"] == 15
    assert h.status_code == 200 and h.json()["loaded_models"] == ["llama-tiny"]
    assert bad.status_code == 400 and bad.json()["message"] == "Model name and prompt are required"
    assert late.status_code == 408
    auth_app = create_worker_app(settings(tmp_path, auth_enabled=True, auth_key="k"),
                                 device="cpu", engine_kwargs=SMALL)
    auth_app.extensions["dli_worker"].load_model("llama-tiny")
    aapp = create_asgi_app(auth_app)

    async def run_auth():
        async with httpx.AsyncClient(transport=httpx.ASGITransport(app=aapp),
                                     base_url="http://w") as c:
            return (await c.post("/inference", json=body),
                    await c.post("/inference", json=body, headers={"Authorization": "Bearer k"}))
    no, yes = asyncio.run(run_auth())
    assert no.status_code == 401 and yes.status_code == 200


def test_master_asgi_long_poll(tmp_path):
    """serve-master --server uvicorn: ?wait= long polls answer on completion (no thread held);
    plain status / pages go through the Flask app."""
    import asyncio
    import httpx
    from distributed_llm_inferencing_amd.control.asgi import create_asgi_app
    w = Server(create_worker_app(settings(tmp_path), device="cpu", engine_kwargs=SMALL))
    flask_app = create_master_app(settings(tmp_path), start_background=True, dispatch_workers=4,
                                  health_interval=0.5)
    app = create_asgi_app(flask_app)

    async def run():
        async with httpx.AsyncClient(transport=httpx.ASGITransport(app=app),
                                     base_url="http://m", timeout=120) as c:
            r = await c.post("/api/nodes/add/", data={"hostname": "cpu0",
                                                      "ip_address": "127.0.0.1", "port": w.port})
            assert r.json()["status"] == "success"
            rid = (await c.post("/api/inference/submit/", data={
                "model_name": "gpt2-tiny", "prompt": "Hello"})).json()["request_id"]
            now = (await c.get(f"/api/inference/status/{rid}/")).json()
            done = (await c.get(f"/api/inference/status/{rid}/", params={"wait": 60})).json()
            missing = await c.get("/api/inference/status/99999/", params={"wait": 1})
            page = await c.get("/")
            return now, done, missing, page
    try:
        now, done, missing, page = asyncio.run(run())
    finally:
        flask_app.extensions["dli"].shutdown()
        w.close()
    assert now["status"] in ("pending", "processing", "completed")
    assert done["status"] == "completed" and done["result"].startswith("Hello")
    assert missing.status_code == 500 and "No InferenceRequest" in missing.json()["message"]
    assert page.status_code == 200


@pytest.mark.parametrize("server,procs", [("aiohttp", 1), ("uvicorn", 1), ("aiohttp", 3)])
def test_control_plane_capacity_harness(server, procs):
    """serve-master on an ASGI server (the aiohttp C-parser front and uvicorn; 3 aiohttp
    processes on one port and one database, control/peers.py) in front of a fake worker,
    driven by the closed-loop load generator through the public API
    (scripts/bench_control_plane.py): every request completes, the submit and long-poll
    fast paths, the on-loop dispatcher and the cross-process completion fan-out included."""
    import json as _json
    import subprocess
    import sys
    root = Path(__file__).resolve().parents[1]
    port = 8800 + (0 if server == "aiohttp" else 10) + 20 * (procs - 1)
    out = subprocess.run([sys.executable, str(root / "scripts" / "bench_control_plane.py"),
                          "--concurrency", "16", "--requests", "64", "--engine-s", "0.05",
                          "--server", server, "--master-port", str(port),
                          "--worker-port", str(port + 1), "--master-procs", str(procs)],
                         capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-2000:]
    rep = _json.loads(out.stdout.strip().splitlines()[-1])
    assert rep["completed"] == 64 and rep["failed"] == 0, rep
    # no long poll waited for its 2 s re-read: completions reached every process
    assert rep["p99_latency_s"] < 1.5, rep
