"""Command-line entry: ``python -m distributed_llm_inferencing_amd.cli <command>``.

Replaces the reference's ``manage.py`` (runserver / shard_model) and its
docker-compose topology (X6: master + 2 worker containers + redis) with a single-node
launcher for an 8-GPU MI355X box.

    serve-master    [--port 8000]                       Flask master (dashboard + API)
    serve-worker    [--port 5000] [--gpu i]             one worker bound to one GPU (or CPU)
    serve-node      --gpus N [--base-port 5000] [--master URL]
                    one worker process per GPU (--gpu i, port base+i; every GPU stays
                    visible to every worker so a ring formed over them by join-pipeline
                    can map its peers' memory), each registered with the master as a node
    serve-pipeline  --model M [--port 5000] [--shard-dir D]
                    (under torchrun) N-rank layer-sharded pipeline; rank 0 serves the worker
                    API and reports the stages as shards; --shard-dir serves the files
                    `shard-model` exported (rank r <- D/shard_<r>/)
    serve-cluster   --model M --gpus 8 --dp K [--base-port 5000] [--master URL]
                    K data-parallel replicas, each a pipeline of gpus/K stages (SURVEY.md
                    §2.5 "DP replicas"); every replica head registers as a node and the
                    master's dispatcher load-balances across them (least in flight)
    serve-expert    --model mixtral-8x7b --gpus N [--base-port 5000] [--master URL]
                    expert-parallel deployment (BASELINE.json config 5): N ranks, one per
                    GPU, each an HTTP worker on port base+rank holding experts
                    [r E/N, (r+1) E/N) and all attention weights; every rank registers
                    as a node and reports its expert shard, the master balances requests
                    across them, and the ranks' MoE layers exchange rows every step
                    (device mailboxes on one node). Spawns its ranks itself, or runs one
                    rank under torchrun
    shard-model     --model_name M --num_shards N [--output_dir D] [--policy even|hbm|balanced]
    join-pipeline   --model M --shard-dir D --nodes URL0,URL1,... [--rendezvous tcp://H:P]
                    assign shard i of an export to node i over the worker API (/load_shard
                    with a "pipeline" spec): the N worker processes form one RCCL ring and
                    node 0 serves the model
    loadgen         --master URL --model M [--requests N] [--concurrency C | --rate R]
                    end-to-end load through the master API: tokens/s, p50/p99 latency
    bench           ... (bench.py)
"""
from __future__ import annotations

import os
import subprocess
import sys
import time


def node_commands(gpus: int, base_port: int = 5000, preload: str = ""):
    """[(argv, env)] of serve-node's workers: worker i selects GPU i of the operator's
    visibility mask with ``--gpu i`` (the mask, if any, is passed through unchanged, so
    ``HIP_VISIBLE_DEVICES=4,5,6,7 serve-node --gpus 4`` runs on physical GPUs 4-7) and sees
    every GPU of that mask. (Masking each worker down to its own GPU would leave a
    join-pipeline ring over them unable to open its peers' memory: the IPC mailboxes and
    RCCL's P2P path both need the peer device visible.)"""
    out = []
    for i in range(gpus):
        env = dict(os.environ)
        env.update(USE_GPU="1", HSA_ENABLE_IPC_MODE_LEGACY="0")
        cmd = [sys.executable, "-m", "distributed_llm_inferencing_amd.worker.server",
               "--port", str(base_port + i), "--gpu", str(i), "--preload", preload]
        out.append((cmd, env))
    return out


def _serve_node(argv):
    import argparse

    import requests
    ap = argparse.ArgumentParser("dli serve-node")
    ap.add_argument("--gpus", type=int, default=8)
    ap.add_argument("--base-port", type=int, default=5000)
    ap.add_argument("--master", default=None, help="e.g. http://127.0.0.1:8000")
    ap.add_argument("--preload", default="")
    a = ap.parse_args(argv)
    procs = []
    for i, (cmd, env) in enumerate(node_commands(a.gpus, a.base_port, a.preload)):
        procs.append(subprocess.Popen(cmd, env=env))
    if a.master:
        for i in range(a.gpus):
            port = a.base_port + i
            for _ in range(120):
                try:
                    r = requests.post(f"{a.master}/api/nodes/add/",
                                      data={"hostname": f"gpu{i}", "ip_address": "127.0.0.1",
                                            "port": port}, timeout=10)
                    if r.status_code == 200:
                        break
                except requests.RequestException:
                    pass
                time.sleep(1)
    try:
        for p in procs:
            p.wait()
    except KeyboardInterrupt:
        for p in procs:
            p.terminate()


def _serve_pipeline(argv):
    """Run under torchrun: rank 0 = HTTP worker + pipeline head; others = stage loops."""
    import argparse
    import logging
    ap = argparse.ArgumentParser("dli serve-pipeline")
    ap.add_argument("--model", required=True)
    ap.add_argument("--port", type=int, default=5000)
    ap.add_argument("--max-batch", type=int, default=256)
    ap.add_argument("--max-model-len", type=int, default=2048)
    ap.add_argument("--policy", default="balanced")
    ap.add_argument("--shard-dir", default=None,
                    help="serve the weights `shard-model` exported: rank r loads "
                         "<dir>/shard_<r>/model.safetensors (layers from its metadata.json)")
    ap.add_argument("--no-shard-report", action="store_true",
                    help="DP replica: serve the model as a plain node (no shard rows)")
    a = ap.parse_args(argv)
    import torch
    from .config import get_settings
    from .parallel.pipeline import DistributedPipelineEngine
    from .worker.server import WorkerState, create_worker_app
    from .worker.service import PipelineService
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = f"cuda:{local}" if torch.cuda.is_available() else "cpu"
    if torch.cuda.is_available():
        torch.cuda.set_device(local)
    eng = DistributedPipelineEngine(a.model, dev, max_batch=a.max_batch,
                                    max_model_len=a.max_model_len, policy=a.policy,
                                    shard_dir=a.shard_dir)
    eng.warmup()
    if eng.rank != 0:
        eng.serve()
        return
    logging.basicConfig(level=logging.INFO)
    s = get_settings()
    s.use_gpu = torch.cuda.is_available()
    st = WorkerState(s, dev)
    st.pipeline_model = a.model
    ch = eng.channel
    st.data_plane = {"kind": "pipeline", "plane": ch.data_plane, "control": ch.ctrl_kind,
                     "fallback": ch.fallback, "ranks": ch.world}
    st.pipeline_service = PipelineService(eng, name=a.model)
    st.tokenizers[a.model] = eng.head.tok
    st.pipeline_shards = [] if a.no_shard_report else [
        {"model_name": a.model, "shard_id": p.shard_id,
         "path": (os.path.join(a.shard_dir, f"shard_{p.shard_id}") if a.shard_dir
                  else f"rank{p.shard_id}"),
         "metadata": p.to_metadata(a.model, len(eng.plans), eng.cfg.num_layers)}
        for p in eng.plans]
    app = create_worker_app(s, state=st)
    app.run(host="0.0.0.0", port=a.port, threaded=True)


def _register_nodes(master: str, ports, prefix: str, timeout_s: float = 1800.0,
                    alive=lambda: True) -> None:
    """Add each worker (127.0.0.1:port) to the master once it answers (/api/nodes/add/
    probes its /health first, as the reference's add_node does)."""
    import requests
    t0 = time.time()
    for i, port in enumerate(ports):
        while time.time() - t0 < timeout_s and alive():
            try:
                r = requests.post(f"{master}/api/nodes/add/",
                                  data={"hostname": f"{prefix}{i}", "ip_address": "127.0.0.1",
                                        "port": port}, timeout=10)
                if r.status_code == 200:
                    break
            except requests.RequestException:
                pass
            time.sleep(1)


def _serve_expert(argv):
    import argparse
    ap = argparse.ArgumentParser("dli serve-expert")
    ap.add_argument("--model", default="mixtral-8x7b")
    ap.add_argument("--gpus", type=int, default=8)
    ap.add_argument("--base-port", type=int, default=5000)
    ap.add_argument("--master", default=None)
    ap.add_argument("--max-batch", type=int, default=256)
    ap.add_argument("--max-model-len", type=int, default=2048)
    ap.add_argument("--model-dir", default=None,
                    help="exported weights (shard-model output or a HF directory): each rank "
                         "reads all attention tensors and only its own experts' rows")
    a = ap.parse_args(argv)
    from . import launch
    if not launch.under_launcher():
        import threading
        procs = launch.start([sys.executable, "-m", "distributed_llm_inferencing_amd.cli",
                              "serve-expert", *argv], a.gpus)
        if a.master:
            threading.Thread(target=_register_nodes, daemon=True, args=(
                a.master, [a.base_port + r for r in range(a.gpus)], "ep",
                1800.0, lambda: all(p.poll() is None for p in procs))).start()
        return launch.wait(procs)
    return _serve_expert_rank(a)


def _serve_expert_rank(a):
    """One EP rank: engine + lockstep service + the worker HTTP API on base_port + rank."""
    import logging

    import torch
    from .config import get_settings
    from .parallel.expert import ExpertParallelEngine
    from .worker.server import WorkerState, create_worker_app
    from .worker.service import ExpertService
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", rank))
    if os.environ.get("DLI_SAME_DEVICE", "0") == "1":
        local = 0
    cuda = torch.cuda.is_available() and os.environ.get("USE_GPU", "1") != "0"
    if cuda:
        torch.cuda.set_device(local)
    dev = torch.device("cuda", local) if cuda else torch.device("cpu")
    kw = {} if cuda else {"num_blocks": 512, "dtype": torch.float32}
    eng = ExpertParallelEngine(a.model, dev, max_batch=a.max_batch,
                               max_model_len=a.max_model_len, model_dir=a.model_dir, **kw)
    eng.warmup()
    logging.basicConfig(level=logging.INFO)
    s = get_settings()
    s.use_gpu = cuda
    st = WorkerState(s, str(dev))
    st.pipeline_model = a.model
    st.pipeline_service = ExpertService(eng, name=a.model.replace("/", "_"))
    st.tokenizers[a.model] = eng.engine.tokenizer
    st.pipeline_shards = [eng.shard_record(a.model)]
    st.data_plane = {"kind": "expert", "plane": eng.data_plane, "fallback": eng.fallback,
                     "ranks": eng.world, "rank": eng.rank}
    app = create_worker_app(s, state=st)
    app.run(host="0.0.0.0", port=a.base_port + eng.rank, threaded=True)
    return 0


def cluster_plan(gpus: int, dp: int, base_port: int = 5000, rdzv_base: int = 29600):
    """[(replica, visible_devices, http_port, rendezvous_port)] for K pipelines of gpus/K."""
    if dp < 1 or gpus % dp:
        raise ValueError(f"--gpus {gpus} is not divisible into {dp} replicas")
    g = gpus // dp
    return [(j, ",".join(str(j * g + i) for i in range(g)), base_port + j, rdzv_base + j)
            for j in range(dp)]


def _serve_cluster(argv):
    import argparse

    import requests
    ap = argparse.ArgumentParser("dli serve-cluster")
    ap.add_argument("--model", required=True)
    ap.add_argument("--gpus", type=int, default=8)
    ap.add_argument("--dp", type=int, default=1)
    ap.add_argument("--base-port", type=int, default=5000)
    ap.add_argument("--master", default=None)
    ap.add_argument("--max-batch", type=int, default=256)
    a, extra = ap.parse_known_args(argv)
    procs = []
    plan = cluster_plan(a.gpus, a.dp, a.base_port)
    for j, devs, port, rdzv in plan:
        env = dict(os.environ, HIP_VISIBLE_DEVICES=devs, USE_GPU="1",
                   HSA_ENABLE_IPC_MODE_LEGACY="0")
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
               f"--nproc-per-node={len(devs.split(','))}", "--master-addr", "127.0.0.1",
               "--master-port", str(rdzv), "-m", "distributed_llm_inferencing_amd.cli",
               "serve-pipeline", "--model", a.model, "--port", str(port),
               "--max-batch", str(a.max_batch), "--no-shard-report", *extra]
        procs.append(subprocess.Popen(cmd, env=env))
    if a.master:
        for j, _devs, port, _ in plan:
            for _ in range(600):
                try:
                    r = requests.post(f"{a.master}/api/nodes/add/",
                                      data={"hostname": f"replica{j}", "ip_address": "127.0.0.1",
                                            "port": port}, timeout=10)
                    if r.status_code == 200:
                        break
                except requests.RequestException:
                    pass
                time.sleep(1)
    try:
        for p in procs:
            p.wait()
    except KeyboardInterrupt:
        for p in procs:
            p.terminate()


def _join_pipeline(argv):
    import argparse
    import json

    import requests
    ap = argparse.ArgumentParser("dli join-pipeline")
    ap.add_argument("--model", required=True)
    ap.add_argument("--shard-dir", required=True, help="<output_dir>/<model> of shard-model")
    ap.add_argument("--nodes", required=True, help="comma-separated worker URLs, stage order")
    ap.add_argument("--rendezvous", default="tcp://127.0.0.1:29650")
    ap.add_argument("--auth-key", default=os.environ.get("AUTH_KEY", ""))
    ap.add_argument("--timeout", type=float, default=600.0)
    a = ap.parse_args(argv)
    nodes = [u.rstrip("/") for u in a.nodes.split(",") if u]
    hdr = {"Authorization": f"Bearer {a.auth_key}"} if a.auth_key else {}
    spec = {"init_method": a.rendezvous, "world_size": len(nodes)}
    for i, u in enumerate(nodes):
        r = requests.post(f"{u}/load_shard", headers=hdr, timeout=30, json={
            "model_name": a.model, "shard_id": i, "pipeline": spec,
            "shard_path": os.path.join(a.shard_dir, f"shard_{i}")})
        print(f"{u}: {r.status_code} {r.json().get('message')}")
        if r.status_code != 200:
            return 1
    t0 = time.time()
    while time.time() - t0 < a.timeout:
        pipes = [requests.get(f"{u}/health", headers=hdr, timeout=10).json()
                 .get("pipeline", {}) for u in nodes]
        states = [p.get("state") for p in pipes]
        if all(s == "serving" for s in states):
            print(json.dumps({"model": a.model, "stages": len(nodes), "head": nodes[0],
                              "data_plane": [p.get("data_plane") for p in pipes],
                              "fallback": [p.get("data_plane_fallback") for p in pipes]}))
            return 0
        if "failed" in states:
            print(f"join failed: {states}: {[p.get('error') for p in pipes]}")
            return 1
        time.sleep(1)
    print(f"join timed out: {states}")
    return 1


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    if not argv or argv[0] in ("-h", "--help"):
        print(__doc__)
        return 0
    cmd, rest = argv[0], argv[1:]
    if cmd == "serve-master":
        from .control.master import main as m
        return m(rest)
    if cmd == "serve-worker":
        from .worker.server import main as m
        return m(rest)
    if cmd == "serve-node":
        return _serve_node(rest)
    if cmd == "serve-pipeline":
        return _serve_pipeline(rest)
    if cmd == "serve-cluster":
        return _serve_cluster(rest)
    if cmd == "serve-expert":
        return _serve_expert(rest)
    if cmd == "shard-model":
        from .shard.writer import main as m
        return m(rest)
    if cmd == "join-pipeline":
        return _join_pipeline(rest)
    if cmd == "loadgen":
        from .loadgen import main as m
        return m(rest)
    if cmd == "bench":
        root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        return subprocess.call([sys.executable, os.path.join(root, "bench.py"), *rest])
    print(f"unknown command {cmd}\n{__doc__}")
    return 2


if __name__ == "__main__":
    sys.exit(main())
