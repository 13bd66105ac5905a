"""Serving the sharded pipeline (CPU, gloo):

* an 8-rank ring serves the per-stage files the ``shard-model`` CLI wrote (each rank
  streams ``shard_<rank>/model.safetensors`` through the C++ loader; with the vocab-parallel
  head every rank reads its row slice of the LM head from the last shard), token-identical
  to the single-stage engine (reference: shard_model.py:94-109 -> worker/app.py:139-206 ->
  master/dashboard/views.py:318-355, which never actually ran more than shard 0);
* continuous admission: requests submitted while a ring session is running join it at the
  next tick and finish before the first session's stragglers (one session in total);
* the worker's ``shard_ids`` path batches concurrent requests (shared decode steps);
* ``/load_model`` reads weights from MODEL_CACHE_DIR (reference worker/app.py:117-124).
"""
import os
import socket
import threading
import time

import pytest
import torch
import torch.multiprocessing as mp

from distributed_llm_inferencing_amd.engine import SamplingParams
from distributed_llm_inferencing_amd.engine.llm_engine import LLMEngine

PROMPTS = [[5, 6, 7, 8], [9, 10, 11], [1, 2, 3, 4, 5, 6, 7], [100, 200], [7] * 9, [3, 4]]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _spawn(target, world, *args):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, q, *args)) for r in range(world)]
    for p in procs:
        p.start()
    return q, procs


def _join(procs):
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0


# ----------------------------------------------------------------------------- shard files
def _shard_worker(rank, world, port, q, shard_root):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank), DLI_PP_VOCAB_PARALLEL="auto")
    torch.set_num_threads(1)
    import torch.distributed as dist
    from distributed_llm_inferencing_amd.parallel.pipeline import DistributedPipelineEngine
    eng = DistributedPipelineEngine("ignored", "cpu", max_batch=8, max_model_len=64,
                                    num_blocks=256, dtype=torch.float32, shard_dir=shard_root)
    if rank == 0:
        sp = SamplingParams(max_length=20, do_sample=False, ignore_eos=True)
        sp2 = SamplingParams(max_length=20, seed=3, ignore_eos=True)
        res = ([o.all_ids for o in eng.generate(PROMPTS, sp)],
               [o.all_ids for o in eng.generate(PROMPTS, sp2)],
               eng.vocab_parallel, [(p.start_layer, p.end_layer) for p in eng.plans],
               eng.channel.ctrl_kind)
        eng.shutdown()
        q.put(res)
    else:
        eng.serve()
    dist.barrier()
    eng.channel.close()
    dist.destroy_process_group()


def test_gloo_ring_serves_shard_files(tmp_path):
    from distributed_llm_inferencing_amd.shard.writer import export_shards, model_dir
    export_shards("llama-tiny8", 8, str(tmp_path), dtype=torch.float32, log=lambda *a: None)
    root = str(model_dir(str(tmp_path), "llama-tiny8"))
    q, procs = _spawn(_shard_worker, 8, root)
    greedy, sampled, vp, plans, ctrl = q.get(timeout=300)
    _join(procs)
    assert vp and ctrl == "shm"
    assert plans == [(i, i + 1) for i in range(8)]          # the files' partition, not ours
    ref = LLMEngine("llama-tiny8", device="cpu", dtype=torch.float32, max_batch=8,
                    max_model_len=64, num_blocks=64)
    assert greedy == [o.all_ids for o in ref.generate(
        PROMPTS, SamplingParams(max_length=20, do_sample=False, ignore_eos=True))]
    assert sampled == [o.all_ids for o in ref.generate(
        PROMPTS, SamplingParams(max_length=20, seed=3, ignore_eos=True))]


# ----------------------------------------------------------------------------- admission
def _admit_worker(rank, world, port, q, vp):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank), DLI_PP_VOCAB_PARALLEL=vp)
    torch.set_num_threads(1)
    import torch.distributed as dist
    from distributed_llm_inferencing_amd.parallel.pipeline import DistributedPipelineEngine
    from distributed_llm_inferencing_amd.worker.service import PipelineService
    eng = DistributedPipelineEngine("llama-tiny", "cpu", max_batch=8, max_model_len=128,
                                    num_blocks=256, dtype=torch.float32)
    if rank != 0:
        eng.serve()
    else:
        svc = PipelineService(eng, name="pp")
        long_sp = SamplingParams(max_length=90, do_sample=False, ignore_eos=True)
        short_sp = SamplingParams(max_length=12, do_sample=False, ignore_eos=True)
        M = eng.microbatches
        done = {}

        def track(key, fut):
            fut.add_done_callback(lambda f: done.setdefault(key, (time.perf_counter(),
                                                                  f.result())))
        # one long request per microbatch, arriving one after another (admission goes to
        # the least-loaded microbatch), so every microbatch is decoding when the short
        # requests arrive
        for i in range(M):
            track(("long", i), svc.submit(ADMIT_PROMPTS[i], long_sp))
            while eng.head.stats.decode_steps < 2 * i + 2:  # the session is running
                time.sleep(0.005)
        while eng.head.stats.decode_steps < 2 * M + 6:
            time.sleep(0.005)
        for i in range(2):
            track(("short", i), svc.submit(ADMIT_PROMPTS[M + i], short_sp))
        while len(done) < M + 2:
            time.sleep(0.01)
        while svc.sessions < 1:
            time.sleep(0.01)
        time.sleep(0.2)
        res = {k: (t, o.all_ids) for k, (t, o) in done.items()}
        q.put((res, svc.sessions, eng.head.sched.num_mixed, M, eng.vocab_parallel))
        svc.close()
        eng.shutdown()
    dist.barrier()
    eng.channel.close()
    dist.destroy_process_group()


ADMIT_PROMPTS = PROMPTS + [[11, 12, 13, 14, 15], [42] * 6, [8, 9]]


@pytest.mark.parametrize("vp", ["0", "1"])
def test_pipeline_service_admits_requests_into_running_session(vp):
    """Requests arriving mid-session join it; they are prefilled in MIXED steps (the
    running microbatch's decode rows ride along; header word 9 tells every stage where the
    decode rows end), with the tail LM head and with the vocab-parallel head; greedy
    tokens equal the single-stage engine's."""
    q, procs = _spawn(_admit_worker, 2, vp)
    res, sessions, mixed, M, vp_on = q.get(timeout=300)
    _join(procs)
    assert vp_on == (vp == "1")
    assert sessions == 1                                   # the late requests joined it
    assert mixed >= 1
    last_long = max(t for (kind, _), (t, _) in res.items() if kind == "long")
    assert all(t < last_long for (kind, _), (t, _) in res.items() if kind == "short")
    ref = LLMEngine("llama-tiny", device="cpu", dtype=torch.float32, max_batch=8,
                    max_model_len=128, num_blocks=128)
    longs = [o.all_ids for o in ref.generate(ADMIT_PROMPTS[:M], SamplingParams(
        max_length=90, do_sample=False, ignore_eos=True))]
    shorts = [o.all_ids for o in ref.generate(ADMIT_PROMPTS[M:M + 2], SamplingParams(
        max_length=12, do_sample=False, ignore_eos=True))]
    assert [res[("long", i)][1] for i in range(M)] == longs
    assert [res[("short", i)][1] for i in range(2)] == shorts


# ----------------------------------------------------------------------------- worker paths
def _settings(tmp_path):
    from distributed_llm_inferencing_amd.config import Settings
    s = Settings()
    s.master_db = str(tmp_path / "db.sqlite3")
    s.model_cache_dir = str(tmp_path / "cache")
    return s


SMALL = dict(max_batch=8, max_model_len=128, num_blocks=256)


def test_worker_sharded_requests_share_decode_steps(tmp_path):
    from distributed_llm_inferencing_amd.shard.writer import export_shards
    from distributed_llm_inferencing_amd.worker.server import create_worker_app
    app = create_worker_app(_settings(tmp_path), device="cpu", engine_kwargs=SMALL)
    c = app.test_client()
    paths = export_shards("llama-tiny", 2, str(tmp_path / "shards"), log=lambda *a: None)
    for i, p in enumerate(paths):
        assert c.post("/load_shard", json={"model_name": "llama-tiny", "shard_id": i,
                                           "shard_path": str(p)}).status_code == 200
    out = [None] * 6

    def call(i):
        out[i] = c.post("/inference", json={"model_name": "llama-tiny", "prompt": f"req {i}",
                                            "max_length": 30, "shard_ids": [0, 1],
                                            "temperature": 0})
    ts = [threading.Thread(target=call, args=(i,)) for i in range(6)]
    [t.start() for t in ts]
    [t.join() for t in ts]
    assert all(r.status_code == 200 for r in out), [r.get_json() for r in out]
    svc = app.extensions["dli_worker"].shard_pipes[("llama-tiny", (0, 1))]
    st = svc.engine.stats
    assert st.finished == 6
    # 6 requests x ~24 new tokens each: serialized would be ~6 x 24 decode steps
    assert st.decode_steps < 3 * 24, st.decode_steps
    single = c.post("/inference", json={"model_name": "llama-tiny", "prompt": "req 0",
                                        "max_length": 30, "temperature": 0}).get_json()
    assert out[0].get_json()["result"] == single["result"]


def test_load_model_reads_model_cache(tmp_path):
    from distributed_llm_inferencing_amd.shard.writer import export_shards
    from distributed_llm_inferencing_amd.worker.server import create_worker_app
    s = _settings(tmp_path)
    # a cache entry with weights that differ from the random init (seed 7)
    export_shards("llama-tiny", 2, s.model_cache_dir, seed=7, dtype=torch.float32,
                  log=lambda *a: None)
    app = create_worker_app(s, device="cpu", engine_kwargs=SMALL)
    c = app.test_client()
    assert c.post("/load_model", json={"model_name": "llama-tiny"}).status_code == 200
    st = app.extensions["dli_worker"]
    assert st.weights_source["llama-tiny"] == "cache"
    body = {"model_name": "llama-tiny", "prompt": "abc", "max_length": 16, "temperature": 0}
    got = c.post("/inference", json=body).get_json()["result"]
    ref = LLMEngine("llama-tiny", device="cpu", dtype=torch.float32, seed=7, max_batch=8,
                    max_model_len=128, num_blocks=64)
    want = ref.generate(["abc"], SamplingParams(max_length=16, temperature=0))[0]
    assert got == want.resolve_text()
    rnd = LLMEngine("llama-tiny", device="cpu", dtype=torch.float32, seed=0, max_batch=8,
                    max_model_len=128, num_blocks=64)
    assert rnd.generate(["abc"], SamplingParams(max_length=16, temperature=0))[0].all_ids \
        != want.all_ids                                   # really not the default init


def _wait_http(url, timeout=120):
    import requests
    t0 = time.time()
    while time.time() - t0 < timeout:
        try:
            return requests.get(url, timeout=2).json()
        except Exception:  # noqa: BLE001
            time.sleep(0.3)
    raise TimeoutError(url)


def test_load_shard_joins_pipeline_ring(tmp_path):
    """W5: two independently started worker processes receive /load_shard with a
    "pipeline" spec, rendezvous (gloo here, RCCL on GPUs) and serve the exported shards as
    one 2-stage ring; requests go to the stage-0 node, which reports both shards; unloading
    the model there shuts the ring down on both nodes."""
    import subprocess
    import sys

    import requests
    from distributed_llm_inferencing_amd.shard.writer import export_shards
    from distributed_llm_inferencing_amd.worker.server import create_worker_app
    paths = export_shards("llama-tiny", 2, str(tmp_path / "shards"), dtype=torch.float32,
                          log=lambda *a: None)
    ports = [_free_port(), _free_port()]
    rdv = _free_port()
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", USE_GPU="0",
               OMP_NUM_THREADS="2", MODEL_CACHE_DIR=str(tmp_path / "cache"))
    procs = [subprocess.Popen([sys.executable, "-m", "distributed_llm_inferencing_amd.worker.server",
                               "--host", "127.0.0.1", "--port", str(p)], env=env,
                              stdout=subprocess.DEVNULL,
                              stderr=open(tmp_path / f"worker{p}.log", "w"))
             for p in ports]
    try:
        urls = [f"http://127.0.0.1:{p}" for p in ports]
        for u in urls:
            _wait_http(f"{u}/health")
        # a repeated /load_shard of the same stage is idempotent; join-pipeline (the CLI the
        # operator uses) assigns shard i to node i and waits for every stage to serve
        from distributed_llm_inferencing_amd.cli import main as cli_main
        spec = {"init_method": f"tcp://127.0.0.1:{rdv}", "world_size": 2}
        r = requests.post(f"{urls[1]}/load_shard", json={
            "model_name": "llama-tiny", "shard_id": 1, "shard_path": str(paths[1]),
            "pipeline": spec}, timeout=30)
        assert r.status_code == 200 and r.json()["pipeline"]["state"] == "joining", r.text
        assert cli_main(["join-pipeline", "--model", "llama-tiny", "--shard-dir",
                         str(paths[0].parent), "--nodes", ",".join(urls), "--rendezvous",
                         spec["init_method"], "--timeout", "240"]) == 0
        hs = [requests.get(f"{u}/health", timeout=5).json() for u in urls]
        states = [h["pipeline"]["state"] for h in hs]
        assert states == ["serving", "serving"], hs
        # every stage reports the data plane its ring resolved (CPU ranks: gloo)
        assert [h["pipeline"]["data_plane"] for h in hs] == ["torch-gloo"] * 2
        assert all(h["data_plane"]["plane"] == "torch-gloo" for h in hs)
        assert sorted(s["shard_id"] for s in hs[0]["loaded_shards"]) == [0, 1]
        assert hs[1]["loaded_shards"] == []   # the master routes this model to stage 0
        body = {"model_name": "llama-tiny", "prompt": "pipeline join", "max_length": 24,
                "temperature": 0, "shard_ids": [0, 1]}
        r0 = requests.post(f"{urls[0]}/inference", json=body, timeout=120)
        assert r0.status_code == 200, r0.text
        assert requests.post(f"{urls[1]}/inference", json=body, timeout=30).status_code == 409
        # same shards through the single-process loopback path
        app = create_worker_app(_settings(tmp_path), device="cpu")
        c = app.test_client()
        for i, p in enumerate(paths):
            c.post("/load_shard", json={"model_name": "llama-tiny", "shard_id": i,
                                        "shard_path": str(p)})
        ref = c.post("/inference", json=body).get_json()
        assert r0.json()["result"] == ref["result"]
        assert requests.post(f"{urls[0]}/unload_model", json={"model_name": "llama-tiny"},
                             timeout=60).status_code == 200
        t0 = time.time()
        while requests.get(f"{urls[1]}/health", timeout=5).json()["pipeline"]["state"] \
                != "stopped":
            assert time.time() - t0 < 60
            time.sleep(0.3)
    finally:
        for p in procs:
            p.terminate()
        for p in procs:
            p.wait(timeout=30)
