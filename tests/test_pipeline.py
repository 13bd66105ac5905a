"""Pipeline parallelism: loopback (single process) and real multi-process rings over gloo
must produce exactly the single-stage engine's tokens."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from distributed_llm_inferencing_amd.engine import SamplingParams
from distributed_llm_inferencing_amd.engine.llm_engine import LLMEngine
from distributed_llm_inferencing_amd.parallel.pipeline import LocalPipeline
from distributed_llm_inferencing_amd.shard.planner import even_split, plan_stages
from distributed_llm_inferencing_amd.models import get_config

PROMPTS = [[5, 6, 7, 8], [9, 10, 11], [1, 2, 3, 4, 5, 6, 7], [100, 200], [7] * 9, [3, 4], [8] * 3]


def _ref(model, sp):
    eng = LLMEngine(model, device="cpu", dtype=torch.float32, max_batch=8, max_model_len=64,
                    num_blocks=64)
    return [o.all_ids for o in eng.generate(PROMPTS, sp)]


@pytest.mark.parametrize("model", ["llama-tiny", "gpt2-tiny", "mixtral-tiny"])
@pytest.mark.parametrize("n", [2, 4])
def test_loopback_pipeline_matches_single_stage(model, n):
    cfg = get_config(model)
    if n > cfg.num_layers:
        pytest.skip("more stages than layers")
    for sp in (SamplingParams(max_length=20, do_sample=False, ignore_eos=True),
               SamplingParams(max_length=20, seed=11, ignore_eos=True)):
        pp = LocalPipeline(model, n, device="cpu", dtype=torch.float32, max_batch=8,
                           max_model_len=64, num_blocks=64)
        assert [o.all_ids for o in pp.generate(PROMPTS, sp)] == _ref(model, sp)


def test_planner_rules():
    assert even_split(32, 3) == [(0, 10), (10, 20), (20, 32)]          # reference rule
    assert even_split(12, 4) == [(0, 3), (3, 6), (6, 9), (9, 12)]
    cfg = get_config("llama3-70b")
    for pol in ("even", "hbm", "balanced"):
        plans = plan_stages(cfg, 8, pol)
        assert plans[0].start_layer == 0 and plans[-1].end_layer == 80
        assert all(a.end_layer == b.start_layer for a, b in zip(plans, plans[1:]))
        assert max(p.weight_bytes for p in plans) < 288 * 2**30
    bal = plan_stages(get_config("llama3-8b"), 8, "balanced")
    # the LM-head stage carries fewer layers
    assert bal[-1].end_layer - bal[-1].start_layer < bal[0].end_layer - bal[0].start_layer
    plan_stages(cfg, 1, "even")                # 70B bf16 (141 GB) fits one 288 GB MI355X
    with pytest.raises(ValueError):            # ...but not a 96 GB device
        plan_stages(cfg, 1, "even", hbm_bytes=96 * 2**30)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


MANY = [[3 + (7 * i + j) % 200 for j in range(4 + i % 5)] for i in range(96)]


def _worker(rank, world, port, model, q, vp="auto"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank), DLI_PP_VOCAB_PARALLEL=vp)
    torch.set_num_threads(1)
    import torch.distributed as dist
    from distributed_llm_inferencing_amd.parallel.pipeline import DistributedPipelineEngine
    eng = DistributedPipelineEngine(model, "cpu", max_batch=8, max_model_len=64, num_blocks=256,
                                    dtype=torch.float32)
    if rank == 0:
        res = []
        for sp in (SamplingParams(max_length=20, do_sample=False, ignore_eos=True),
                   SamplingParams(max_length=20, seed=11, ignore_eos=True)):
            res.append([o.all_ids for o in eng.generate(PROMPTS, sp)])
        # a second session on the same ring (sessions start/stop cleanly)
        res.append([o.all_ids for o in eng.generate(PROMPTS[:2], SamplingParams(
            max_length=12, do_sample=False, ignore_eos=True))])
        # top_k = 0 (full-vocabulary top-p) falls back to the tail's LM head per step
        res.append([o.all_ids for o in eng.generate(PROMPTS[:3], SamplingParams(
            max_length=16, top_k=0, top_p=0.9, seed=5, ignore_eos=True))])
        res.append(eng.vocab_parallel)
        if world >= 8:
            # every microbatch full for many ticks: the head's control-plane backlog to the
            # far stages is deepest here (a blocking drain before the exchange deadlocked)
            res.append([o.all_ids for o in eng.generate(MANY, SamplingParams(
                max_length=28, do_sample=False, ignore_eos=True))])
        eng.shutdown()
        q.put(res)
    else:
        eng.serve()
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,vp", [(2, "0"), (3, "0"), (2, "1"), (4, "auto"), (8, "auto")])
def test_gloo_ring_matches_single_stage(world, vp):
    """Pipeline over gloo ranks == single-stage engine, token for token (greedy, sampled,
    second session, full-vocab fallback), with the tail LM head and with the vocab-parallel
    head (every rank scores 1/N of the vocabulary; rank 0 samples from the candidates)."""
    model = "llama-tiny"
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, model, q, vp))
             for r in range(world)]
    for p in procs:
        p.start()
    res = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    greedy = SamplingParams(max_length=20, do_sample=False, ignore_eos=True)
    assert res[0] == _ref(model, greedy)
    assert res[1] == _ref(model, SamplingParams(max_length=20, seed=11, ignore_eos=True))
    eng = LLMEngine(model, device="cpu", dtype=torch.float32, max_batch=8, max_model_len=64,
                    num_blocks=64)
    assert res[2] == [o.all_ids for o in eng.generate(PROMPTS[:2], SamplingParams(
        max_length=12, do_sample=False, ignore_eos=True))]
    assert res[3] == [o.all_ids for o in eng.generate(PROMPTS[:3], SamplingParams(
        max_length=16, top_k=0, top_p=0.9, seed=5, ignore_eos=True))]
    assert res[4] == (vp == "1" or (vp == "auto" and world >= 4))
    if world >= 8:
        assert res[5] == [o.all_ids for o in eng.generate(MANY, SamplingParams(
            max_length=28, do_sample=False, ignore_eos=True))]


def _ep_worker(rank, world, port, q, model, bound_max):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      DLI_EP_BOUND_MAX_TOKENS=str(bound_max))
    torch.set_num_threads(1)
    import torch.distributed as dist
    from distributed_llm_inferencing_amd.parallel.expert import ExpertParallelEngine
    eng = ExpertParallelEngine(model, "cpu", max_batch=8, max_model_len=64,
                               num_blocks=64, dtype=torch.float32)
    # ranks serve DIFFERENT requests (DP attention) and unequal amounts (idle-step path)
    mine = PROMPTS[rank::world] if rank == 0 else PROMPTS[rank::world][:1]
    sp = SamplingParams(max_length=18, do_sample=False, ignore_eos=True)
    out = [o.all_ids for o in eng.generate(mine, sp)]
    st = eng.engine.stats
    q.put((rank, mine, out, eng.moe.exchanges, eng.moe.host_reads, eng.lockstep_syncs,
           eng.steps, st.prefill_steps, eng.engine.lookahead))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("model,world,bound_max", [("mixtral-tiny", 2, 1024),
                                                   ("mixtral-tiny", 4, 1024),
                                                   ("mixtral-tiny8e", 8, 1024),
                                                   ("mixtral-tiny8e", 4, 4)])
def test_expert_parallel_gloo_matches_dense(model, world, bound_max):
    """DP attention + EP experts over gloo ranks == single process with all experts, with
    lookahead on. Routing never reaches the host on a decode step: the only host syncs are
    the one lockstep exchange per step (plus, with the exact-count path forced on steps
    above ``bound_max`` tokens, one read per MoE layer of those prefill steps)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ep_worker, args=(r, world, port, q, model, bound_max))
             for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    eng = LLMEngine(model, device="cpu", dtype=torch.float32, max_batch=8,
                    max_model_len=64, num_blocks=64)
    sp = SamplingParams(max_length=18, do_sample=False, ignore_eos=True)
    L = get_config(model).num_layers
    for rank, mine, out, exch, reads, syncs, steps, prefills, la in res:
        assert out == [o.all_ids for o in eng.generate(mine, sp)], rank
        assert exch == steps * L and la                 # lockstep forwards, lookahead on
        assert syncs == steps + 1                       # one exchange per step (+ the last)
        if bound_max >= 64:
            assert reads == 0                           # no routing read on any step
    # every rank ran the same exchanges; the exact path read counts on prefill steps only
    assert len({r[3] for r in res}) == 1 and len({r[4] for r in res}) == 1
    if bound_max < 64:
        assert 0 < res[0][4] <= L * max(r[7] for r in res)


def _tp_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    import torch.distributed as dist
    from distributed_llm_inferencing_amd.parallel.tensor import TensorParallelEngine
    eng = TensorParallelEngine("llama-tiny", "cpu", max_batch=8, max_model_len=64,
                               num_blocks=64, dtype=torch.float32)
    greedy = SamplingParams(max_length=16, do_sample=False, ignore_eos=True)
    sampled = SamplingParams(max_length=16, seed=5, ignore_eos=True)
    out = ([o.all_ids for o in eng.generate(PROMPTS[:3], greedy)],
           [o.all_ids for o in eng.generate(PROMPTS[:3], sampled)])
    q.put((rank, out, eng.reduce.calls, eng.engine.cfg.num_kv_heads))
    dist.barrier()
    dist.destroy_process_group()


def test_tensor_parallel_gloo_matches_dense():
    """Head/FFN-sharded layers + all-reduce over 2 gloo ranks == the unsharded model."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_tp_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    eng = LLMEngine("llama-tiny", device="cpu", dtype=torch.float32, max_batch=8,
                    max_model_len=64, num_blocks=64)
    greedy = [o.all_ids for o in eng.generate(PROMPTS[:3], SamplingParams(
        max_length=16, do_sample=False, ignore_eos=True))]
    assert res[0][1][0] == greedy and res[1][1][0] == greedy
    assert res[0][1][1] == res[1][1][1]            # ranks agree on sampled tokens
    assert res[0][2] > 0 and res[0][3] == 1        # 2 kv heads split over 2 ranks


def _dying_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank), DLI_PP_VOCAB_PARALLEL="0",
                      DLI_PP_TIMEOUT_S="60")
    if rank == 1:
        os.environ["DLI_FAULT"] = "pipeline.stage:exit_after:6"   # dies on its 7th tick
    torch.set_num_threads(1)
    import time
    from distributed_llm_inferencing_amd.parallel.pipeline import DistributedPipelineEngine
    from distributed_llm_inferencing_amd.worker.service import PipelineService
    eng = DistributedPipelineEngine("llama-tiny", "cpu", max_batch=8, max_model_len=64,
                                    num_blocks=256, dtype=torch.float32)
    if rank != 0:
        eng.serve()                   # never returns: the fault hard-exits this process
        return
    svc = PipelineService(eng, name="pp")
    t0 = time.perf_counter()
    sp = SamplingParams(max_length=30, do_sample=False, ignore_eos=True)
    err = None
    try:
        svc.generate(PROMPTS[0], sp, timeout=120)
    except Exception as e:  # noqa: BLE001
        err = repr(e)
    later = None
    try:
        svc.generate(PROMPTS[1], sp, timeout=5)
    except Exception as e:  # noqa: BLE001
        later = repr(e)
    q.put((err, later, svc.error is not None, time.perf_counter() - t0))
    q.close()
    q.join_thread()                   # flush the queue before the hard exit below
    os._exit(0)                       # the ring is gone: no collective teardown possible


def test_pipeline_stage_death_fails_fast_and_marks_unhealthy():
    """SURVEY.md §5.3 failure detection: a stage process that dies mid-session (injected
    hard exit) turns into an error on the head within the data-plane timeout — not a hang —
    the pending request fails, later requests fail immediately, and the service reports the
    failure (the worker's /health then answers 503)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_dying_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    err, later, failed, dt = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
    assert procs[1].exitcode == 17                       # the injected stage death
    assert err is not None and later is not None and failed
    assert "failed" in later
    assert dt < 120
