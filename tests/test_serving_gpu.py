"""Multi-process serving on the GPU, every rank on cuda:0 (``DLI_SAME_DEVICE=1``: the box
has one MI355X): the deployments the driver's 8-GPU node would run, with the data plane
each one resolves reported by the workers themselves.

* ``serve-worker`` x 2 + ``join-pipeline``: a 2-stage ring formed over the worker API
  (``/load_shard`` with a pipeline spec) must resolve to the device mailboxes (``ipc``)
  with no data-plane override, and answer like the single-process loopback pipeline;
* ``serve-expert``: 2 EP ranks registered with the master, requests submitted through
  ``/api/inference/submit/``, token-identical to one engine holding every expert.
"""
from __future__ import annotations

import os
import signal
import socket
import subprocess
import sys
import time
from pathlib import Path

import pytest
import requests
import torch

from distributed_llm_inferencing_amd.engine import SamplingParams
from distributed_llm_inferencing_amd.engine.llm_engine import LLMEngine

from test_control_plane import Server, settings

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[1]


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _two_ports() -> int:
    while True:
        base = _free_port()
        try:
            with socket.socket() as s:
                s.bind(("127.0.0.1", base + 1))
            return base
        except OSError:
            continue


def _wait(pred, timeout, what):
    t0 = time.time()
    while time.time() - t0 < timeout:
        try:
            v = pred()
        except requests.RequestException:
            v = None
        if v:
            return v
        time.sleep(0.3)
    raise AssertionError(f"timed out waiting for {what}")


def _env(**kw):
    env = dict(os.environ, DLI_SAME_DEVICE="1", DLI_GEMM_AUTOTUNE="0", USE_GPU="1",
               PYTHONPATH=str(ROOT), **kw)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "DLI_PP_COMM", "DLI_EP_COMM",
              "DLI_DIST_BACKEND"):
        env.pop(k, None)
    return env


def _stop(procs):
    for p in procs:
        if p.poll() is None:
            p.send_signal(signal.SIGTERM)
    for p in procs:
        try:
            p.wait(timeout=60)
        except subprocess.TimeoutExpired:
            p.kill()
            p.wait()


@pytest.mark.timeout(600)
def test_join_pipeline_over_two_workers_resolves_ipc(gpu, tmp_path):
    from distributed_llm_inferencing_amd.cli import main as cli_main
    from distributed_llm_inferencing_amd.shard.writer import export_shards
    from distributed_llm_inferencing_amd.worker.server import create_worker_app
    paths = export_shards("llama-tiny", 2, str(tmp_path / "shards"), log=lambda *a: None)
    base = _two_ports()
    env = _env(MODEL_CACHE_DIR=str(tmp_path / "cache"))
    procs = [subprocess.Popen([sys.executable, "-m", "distributed_llm_inferencing_amd.worker.server",
                               "--host", "127.0.0.1", "--port", str(base + i), "--gpu", "0",
                               "--max-batch", "8"], env=env, cwd=ROOT,
                              stdout=subprocess.DEVNULL,
                              stderr=open(tmp_path / f"worker{i}.log", "w"))
             for i in range(2)]
    try:
        urls = [f"http://127.0.0.1:{base + i}" for i in range(2)]
        for u in urls:
            _wait(lambda u=u: requests.get(f"{u}/health", timeout=2).json(), 180, u)
        rdv = f"tcp://127.0.0.1:{_free_port()}"
        rc = cli_main(["join-pipeline", "--model", "llama-tiny", "--shard-dir",
                       str(paths[0].parent), "--nodes", ",".join(urls), "--rendezvous", rdv,
                       "--timeout", "300"])
        assert rc == 0, "\n".join((tmp_path / f"worker{i}.log").read_text()[-3000:]
                                  for i in range(2))
        hs = [requests.get(f"{u}/health", timeout=10).json() for u in urls]
        assert [h["pipeline"]["state"] for h in hs] == ["serving", "serving"], hs
        assert [h["pipeline"]["data_plane"] for h in hs] == ["ipc", "ipc"], hs
        assert all("data_plane_fallback" not in h["pipeline"] for h in hs)
        body = {"model_name": "llama-tiny", "prompt": "xGMI ring", "max_length": 24,
                "temperature": 0, "shard_ids": [0, 1]}
        r0 = requests.post(f"{urls[0]}/inference", json=body, timeout=120)
        assert r0.status_code == 200, r0.text
        os.environ["DLI_GEMM_AUTOTUNE"] = "0"        # the ranks' plans: heuristic too
        try:
            app = create_worker_app(settings(tmp_path), device="cuda:0",
                                    engine_kwargs=dict(max_batch=8, max_model_len=128,
                                                       num_blocks=64))
            c = app.test_client()
            for i, p in enumerate(paths):
                c.post("/load_shard", json={"model_name": "llama-tiny", "shard_id": i,
                                            "shard_path": str(p)})
            ref = c.post("/inference", json=body).get_json()["result"]
        finally:
            del os.environ["DLI_GEMM_AUTOTUNE"]
        assert r0.json()["result"] == ref
        assert requests.post(f"{urls[0]}/unload_model", json={"model_name": "llama-tiny"},
                             timeout=60).status_code == 200
    finally:
        _stop(procs)


@pytest.mark.timeout(600)
def test_serve_expert_on_gpu_through_master(gpu, tmp_path):
    from distributed_llm_inferencing_amd.control.master import create_master_app
    master = create_master_app(settings(tmp_path), start_background=True, dispatch_workers=8)
    ms = Server(master)
    base = _two_ports()
    proc = subprocess.Popen([sys.executable, "-m", "distributed_llm_inferencing_amd.cli",
                             "serve-expert", "--model", "mixtral-tiny", "--gpus", "2",
                             "--base-port", str(base), "--master", ms.url, "--max-batch", "8",
                             "--max-model-len", "256"], cwd=ROOT, env=_env(),
                            stdout=subprocess.DEVNULL,
                            stderr=open(tmp_path / "serve_expert.log", "w"))
    prompts = ["Mixtral on MI355X", "experts over xGMI", "hello", "rank balance"]
    try:
        def nodes():
            n = requests.get(f"{ms.url}/api/nodes/status/", timeout=10).json()["nodes"]
            return n if len(n) == 2 and all(x["is_active"] for x in n) else None
        _wait(nodes, 300, "both EP ranks registered")
        for r in range(2):
            h = requests.get(f"http://127.0.0.1:{base + r}/health", timeout=10).json()
            assert h["data_plane"]["plane"] == "ipc" and not h["data_plane"]["fallback"], h
        rids = [requests.post(f"{ms.url}/api/inference/submit/",
                              data={"model_name": "mixtral-tiny", "prompt": p},
                              timeout=10).json()["request_id"] for p in prompts]

        def done():
            st = [requests.get(f"{ms.url}/api/inference/status/{r}/", timeout=10).json()
                  for r in rids]
            return st if all(s["status"] in ("completed", "failed") for s in st) else None
        sts = _wait(done, 300, "requests completed")
        assert all(s["status"] == "completed" for s in sts), sts
        served = [requests.get(f"http://127.0.0.1:{base + r}/metrics", timeout=10).json()
                  ["engines"]["mixtral-tiny"]["finished_requests"] for r in range(2)]
        assert sum(served) == len(prompts) and min(served) > 0, served
        os.environ["DLI_GEMM_AUTOTUNE"] = "0"
        try:
            dense = LLMEngine("mixtral-tiny", device="cuda", max_batch=8, max_model_len=256,
                              num_blocks=64)
            for p, rid, st in zip(prompts, rids, sts):
                ref = dense.generate([p], SamplingParams(max_length=100, temperature=0.8,
                                                         top_k=50, top_p=0.95, seed=rid))[0]
                assert st["result"] == ref.resolve_text(), (p, rid)
        finally:
            del os.environ["DLI_GEMM_AUTOTUNE"]
    finally:
        _stop([proc])
        ms.close()
        master.extensions["dli"].shutdown()
