"""Ring failure recovery and request re-dispatch.

The reference marks a failing node inactive and keeps dispatching to the next active node
(master/dashboard/views.py:99-105,389-391); nothing in it could recover a sharded model. Here,
on CPU with real worker processes and a real master:

1. replica A = a 4-stage layer-sharded ring formed through ``/load_shard`` pipeline specs
   (``dli join-pipeline``); replica B = one worker loading the same exported weights from
   MODEL_CACHE_DIR; both are plain nodes of the master (DP replicas do not report shard
   rows, which the reference keys uniquely by (model, shard id));
2. stage 2 of A hard-exits mid-session (injected ``pipeline.stage:exit_after``): the head
   aborts its ring, answers 503, keeps its process;
3. every request that was in flight on A is re-dispatched by the master to B and completes;
4. a fresh worker replaces stage 2 and ``join-pipeline`` re-forms the ring around the SAME
   head process, which serves again.

The whole test is time-bounded (pytest-timeout + bounded waits)."""
import os
import socket
import subprocess
import sys
import threading
import time

import pytest
import requests
import torch


_USED_PORTS = set()


def _free_port():
    """A free loopback port not handed out before in this process (the OS may return the
    same ephemeral port to two bind(0) calls once the first socket is closed: two stage
    workers on one port made join-pipeline post shard 3 to stage 2's worker)."""
    while True:
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            p = s.getsockname()[1]
        if p not in _USED_PORTS:
            _USED_PORTS.add(p)
            return p


def _wait_http(url, t=120):
    t0 = time.time()
    while time.time() - t0 < t:
        try:
            return requests.get(url, timeout=2)
        except Exception:  # noqa: BLE001
            time.sleep(0.3)
    raise TimeoutError(url)


def _worker(tmp_path, port, extra_env=None):
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", USE_GPU="0",
               OMP_NUM_THREADS="1", MODEL_CACHE_DIR=str(tmp_path / "cache"),
               DLI_PP_TIMEOUT_S="30", DLI_PP_VOCAB_PARALLEL="0", DLI_FAULT="",
               DLI_REPORT_PIPELINE_SHARDS="0")
    env.update(extra_env or {})
    return subprocess.Popen([sys.executable, "-m", "distributed_llm_inferencing_amd.worker.server",
                             "--host", "127.0.0.1", "--port", str(port)], env=env,
                            stdout=subprocess.DEVNULL,
                            stderr=open(tmp_path / f"worker{port}.log", "w"))


class _Server:
    def __init__(self, app):
        from werkzeug.serving import make_server
        self.srv = make_server("127.0.0.1", 0, app, threaded=True)
        self.url = f"http://127.0.0.1:{self.srv.server_port}"
        threading.Thread(target=self.srv.serve_forever, daemon=True).start()

    def close(self):
        self.srv.shutdown()


@pytest.mark.timeout(600)
def test_stage_death_redispatch_and_ring_reform(tmp_path):
    from distributed_llm_inferencing_amd.cli import main as cli_main
    from distributed_llm_inferencing_amd.config import Settings
    from distributed_llm_inferencing_amd.control.master import create_master_app
    from distributed_llm_inferencing_amd.shard.writer import export_shards
    paths = export_shards("llama-tiny", 4, str(tmp_path / "cache"), dtype=torch.float32,
                          log=lambda *a: None)
    shard_dir = str(paths[0].parent)
    ports = [_free_port() for _ in range(4)]
    port_b = _free_port()
    procs = [_worker(tmp_path, p, {"DLI_FAULT": "pipeline.stage:exit_after:60"} if i == 2
                     else None) for i, p in enumerate(ports)]
    procs.append(_worker(tmp_path, port_b))
    urls = [f"http://127.0.0.1:{p}" for p in ports]
    url_b = f"http://127.0.0.1:{port_b}"
    master = None
    ms = None
    try:
        for u in urls + [url_b]:
            _wait_http(f"{u}/health")
        rdv = f"tcp://127.0.0.1:{_free_port()}"
        assert cli_main(["join-pipeline", "--model", "llama-tiny", "--shard-dir", shard_dir,
                         "--nodes", ",".join(urls), "--rendezvous", rdv,
                         "--timeout", "240"]) == 0
        r = requests.post(f"{url_b}/load_model", json={"model_name": "llama-tiny"}, timeout=60)
        assert r.status_code == 200, r.text
        s = Settings()
        s.master_db = str(tmp_path / "m.sqlite3")
        s.model_cache_dir = str(tmp_path / "cache")
        master = create_master_app(s, start_background=True, dispatch_workers=8,
                                   health_interval=0.5)
        ms = _Server(master)
        for host, u in (("ringA", urls[0]), ("replicaB", url_b)):
            port = u.rsplit(":", 1)[1]
            r = requests.post(f"{ms.url}/api/nodes/add/", data={
                "hostname": host, "ip_address": "127.0.0.1", "port": port}, timeout=10)
            assert r.status_code == 200, r.text
        st = master.extensions["dli"]
        rids = []
        for i in range(12):
            r = requests.post(f"{ms.url}/api/inference/submit/",
                              data={"model_name": "llama-tiny", "prompt": f"recover {i} " * 3},
                              timeout=10)
            rids.append(r.json()["request_id"])
        death = {}

        def watch():                       # stage 2's exit -> the head answering 503
            while procs[2].poll() is None:
                time.sleep(0.02)
            death["exit"] = time.time()
            while time.time() - death["exit"] < 60:
                try:
                    if requests.get(f"{urls[0]}/health", timeout=2).status_code == 503:
                        death["503"] = time.time()
                        return
                except Exception:  # noqa: BLE001
                    pass
                time.sleep(0.05)
        threading.Thread(target=watch, daemon=True).start()
        t0 = time.time()
        while True:
            rows = [st.store.get_request(r) for r in rids]
            if all(x["status"] in ("completed", "failed") for x in rows):
                break
            assert time.time() - t0 < 240, [x["status"] for x in rows]
            time.sleep(0.5)
        assert [x["status"] for x in rows] == ["completed"] * 12, rows
        assert procs[2].wait(timeout=60) == 17            # the injected stage death
        # the ring watchdog (stage pid liveness on the control ring) fails the session within
        # ~0.2 s of the death; /health answers 503 well inside the reference's 5 s probe
        t1 = time.time()
        while "503" not in death and time.time() - t1 < 30:
            time.sleep(0.1)
        assert "503" in death and death["503"] - death["exit"] < 5.0, death
        # some requests were retried: their first node was the broken ring
        assert any(int(x.get("attempts") or 1) > 1 for x in rows), rows
        h = requests.get(f"{urls[0]}/health", timeout=10)
        assert h.status_code == 503 and "pipeline failed" in h.json()["message"]
        # a fresh worker replaces stage 2; the same head process re-forms the ring
        port2 = _free_port()
        procs.append(_worker(tmp_path, port2))
        urls2 = [urls[0], urls[1], f"http://127.0.0.1:{port2}", urls[3]]
        _wait_http(f"{urls2[2]}/health")
        rdv2 = f"tcp://127.0.0.1:{_free_port()}"
        assert cli_main(["join-pipeline", "--model", "llama-tiny", "--shard-dir", shard_dir,
                         "--nodes", ",".join(urls2), "--rendezvous", rdv2,
                         "--timeout", "240"]) == 0
        body = {"model_name": "llama-tiny", "prompt": "served again", "max_length": 24,
                "temperature": 0}
        r = requests.post(f"{urls[0]}/inference", json=body, timeout=120)
        assert r.status_code == 200 and r.json()["status"] == "success", r.text
        ref = requests.post(f"{url_b}/inference", json=body, timeout=120)
        assert r.json()["result"] == ref.json()["result"]
        assert requests.get(f"{urls[0]}/health", timeout=10).status_code == 200
    finally:
        if ms is not None:
            ms.close()
        if master is not None:
            master.extensions["dli"].shutdown()
        for p in procs:
            if p.poll() is None:
                p.terminate()
        for p in procs:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                p.kill()
