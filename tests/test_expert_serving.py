"""Expert parallelism served through the worker / master API (BASELINE.json config 5,
"experts mapped to worker shards"): ``cli serve-expert`` starts N EP ranks, each an HTTP
worker registered with the master as a node reporting its expert shard; requests submitted
to ``/api/inference/submit/`` are balanced across the ranks, whose MoE layers exchange rows
every step. Results must be token-identical to one dense engine holding every expert.
Reference flow: master/dashboard/views.py:318-355,389-391 -> worker/app.py:252-330."""
from __future__ import annotations

import os
import signal
import socket
import subprocess
import sys
import time
from pathlib import Path

import requests
import torch

from distributed_llm_inferencing_amd.engine import SamplingParams
from distributed_llm_inferencing_amd.engine.llm_engine import LLMEngine

from test_control_plane import Server, settings

ROOT = Path(__file__).resolve().parents[1]
PROMPTS = ["Mixtral experts", "one MI355X per rank", "xGMI all-to-all", "hello", "shards",
           "expert parallel serving"]


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _wait(pred, timeout, what):
    t0 = time.time()
    while time.time() - t0 < timeout:
        v = pred()
        if v:
            return v
        time.sleep(0.2)
    raise AssertionError(f"timed out waiting for {what}")


def test_serve_expert_through_master_matches_dense(tmp_path):
    from distributed_llm_inferencing_amd.control.master import create_master_app
    master = create_master_app(settings(tmp_path), start_background=True, dispatch_workers=8)
    ms = Server(master)
    # two free ports in a row for the ranks (base, base + 1)
    while True:
        base = _free_port()
        try:
            with socket.socket() as s:
                s.bind(("127.0.0.1", base + 1))
            break
        except OSError:
            continue
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", USE_GPU="0",
               OMP_NUM_THREADS="2", PYTHONPATH=str(ROOT))
    env.pop("WORLD_SIZE", None)
    env.pop("RANK", None)
    proc = subprocess.Popen([sys.executable, "-m", "distributed_llm_inferencing_amd.cli",
                             "serve-expert", "--model", "mixtral-tiny", "--gpus", "2",
                             "--base-port", str(base), "--master", ms.url, "--max-batch", "8",
                             "--max-model-len", "256"], cwd=ROOT, env=env)
    try:
        def nodes():
            n = requests.get(f"{ms.url}/api/nodes/status/", timeout=10).json()["nodes"]
            return n if len(n) == 2 and all(x["is_active"] for x in n) else None
        ns = _wait(nodes, 240, "both EP ranks registered")
        shards = sorted((s for n in ns for s in n.get("loaded_shards", [])),
                        key=lambda s: s["shard_id"])
        assert [s["shard_id"] for s in shards] == [0, 1]
        assert [s["metadata"]["experts"] for s in shards] == [[0, 2], [2, 4]]
        assert all(s["metadata"]["kind"] == "expert" for s in shards)
        for r in range(2):
            h = requests.get(f"http://127.0.0.1:{base + r}/health", timeout=10).json()
            assert h["data_plane"]["kind"] == "expert" and h["data_plane"]["ranks"] == 2
            assert h["data_plane"]["plane"] in ("torch-gloo", "ipc-host")

        rids = [requests.post(f"{ms.url}/api/inference/submit/",
                              data={"model_name": "mixtral-tiny", "prompt": p},
                              timeout=10).json()["request_id"] for p in PROMPTS]

        def done():
            st = [requests.get(f"{ms.url}/api/inference/status/{r}/", timeout=10).json()
                  for r in rids]
            return st if all(s["status"] in ("completed", "failed") for s in st) else None
        sts = _wait(done, 300, "requests completed")
        assert all(s["status"] == "completed" for s in sts), sts

        # both ranks served requests (the master balances across the shard holders)
        served = []
        for r in range(2):
            m = requests.get(f"http://127.0.0.1:{base + r}/metrics", timeout=10).json()
            served.append(m["engines"]["mixtral-tiny"]["finished_requests"])
        assert sum(served) == len(PROMPTS) and min(served) > 0, served

        # token-identical to one engine holding every expert (seed = the master's request id)
        dense = LLMEngine("mixtral-tiny", device="cpu", dtype=torch.float32, max_batch=8,
                          max_model_len=256, num_blocks=512)
        for p, rid, st in zip(PROMPTS, rids, sts):
            sp = SamplingParams(max_length=100, temperature=0.8, top_k=50, top_p=0.95,
                                seed=rid)
            ref = dense.generate([p], sp)[0]
            assert st["result"] == ref.resolve_text(), (p, rid)
    finally:
        proc.send_signal(signal.SIGTERM)
        try:
            proc.wait(timeout=60)
        except subprocess.TimeoutExpired:
            proc.kill()
            proc.wait()
        ms.close()
        master.extensions["dli"].shutdown()
