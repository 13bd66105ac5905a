"""Tag-blind FIFO data plane (parallel/fifo.py, the host model of csrc/runtime/ipc.cpp).

gloo matches point-to-point messages by (peer, tag); RCCL and the device mailboxes match by
issue order per (src, dst) and ignore tags. These tests run every multi-rank schedule
through the shared-memory mailbox transport, which enforces the RCCL rule (and asserts
equal sizes), so an ordering bug that gloo would hide fails here on CPU:

* the transport itself: FIFO per edge, size mismatch detected, mailbox capacity enforced;
* the layer-sharded pipeline at N = 2..8, tail head and vocab-parallel head, mixed steps,
  chunked prefill: token-identical to the single-stage engine.
"""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from distributed_llm_inferencing_amd.engine import SamplingParams
from distributed_llm_inferencing_amd.engine.llm_engine import LLMEngine

PROMPTS = [[5, 6, 7, 8], [9, 10, 11], [1, 2, 3, 4, 5, 6, 7], [100, 200], [7] * 9, [3, 4], [8] * 3]
LONG = [list(range(3, 3 + 40)), [11] * 37]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _env(rank, world, port, **kw):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank), DLI_PP_COMM="ipc", **kw)
    torch.set_num_threads(1)


def _spawn(target, world, *args, n_results=1, timeout=300):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, q) + args) for r in range(world)]
    for p in procs:
        p.start()
    try:
        res = [q.get(timeout=timeout) for _ in range(n_results)]
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    return res


# ------------------------------------------------------------------------------ transport
def _transport_worker(rank, world, port, q):
    _env(rank, world, port)
    import torch.distributed as dist
    dist.init_process_group("gloo")
    from distributed_llm_inferencing_amd.parallel.fifo import (FifoMismatch,
                                                               ShmMailboxTransport, mailbox_caps)
    ep = ShmMailboxTransport(world, rank, mailbox_caps(world, 4096, 4096),
                             f"/dli_fifo_t_{port}", timeout_s=20)
    dist.barrier()
    ep.connect()
    dist.barrier()
    out = {}
    nxt, prv = (rank + 1) % world, (rank - 1) % world
    # FIFO: three messages of different sizes on one edge, received in send order
    msgs = [torch.arange(n, dtype=torch.int32) + 100 * rank for n in (3, 17, 5)]
    got = [torch.empty(n, dtype=torch.int32) for n in (3, 17, 5)]
    for m, g in zip(msgs, got):          # one message per exchange: the mailbox holds one
        ep.exchange([(m, nxt)], [(g, prv)])
    out["fifo"] = all(torch.equal(g, torch.arange(g.numel(), dtype=torch.int32) + 100 * prv)
                      for g in got)
    # order divergence: rank 0 sends 8 then 4 ints, rank 1 receives 4 then 8
    if world == 2:
        try:
            if rank == 0:
                ep.exchange([(torch.zeros(8, dtype=torch.int32), 1)], [])
                ep.exchange([(torch.zeros(4, dtype=torch.int32), 1)], [])
                out["mismatch"] = None
            else:
                ep.exchange([], [(torch.empty(4, dtype=torch.int32), 0)])
                out["mismatch"] = None
        except FifoMismatch as e:
            out["mismatch"] = str(e)
        except TimeoutError as e:
            out["mismatch"] = "timeout: " + str(e)
    try:
        ep.send(torch.zeros(2048, dtype=torch.int32), nxt)
        out["cap"] = None
    except ValueError as e:
        out["cap"] = str(e)
    q.put((rank, out))
    dist.barrier()
    ep.close()
    dist.destroy_process_group()


def test_fifo_transport_orders_and_checks_sizes():
    res = dict(_spawn(_transport_worker, 2, n_results=2))
    assert res[0]["fifo"] and res[1]["fifo"]
    assert "differs between the two ranks" in res[1]["mismatch"]
    assert "exceeds the mailbox" in res[0]["cap"]


# ------------------------------------------------------------------------------ pipeline
def _pp_worker(rank, world, port, q, vp, mixed, chunk, schedule="piped"):
    _env(rank, world, port, DLI_PP_VOCAB_PARALLEL=vp, DLI_MIXED_STEPS=mixed,
         DLI_PP_SCHEDULE=schedule)
    import torch.distributed as dist
    from distributed_llm_inferencing_amd.parallel.pipeline import DistributedPipelineEngine
    eng = DistributedPipelineEngine("llama-tiny", "cpu", max_batch=4, max_model_len=64,
                                    num_blocks=256, dtype=torch.float32,
                                    max_prefill_tokens=chunk)
    assert eng.channel.ipc is not None
    if rank == 0:
        res = []
        greedy = SamplingParams(max_length=20, do_sample=False, ignore_eos=True)
        res.append([o.all_ids for o in eng.generate(PROMPTS, greedy)])
        res.append([o.all_ids for o in eng.generate(PROMPTS, SamplingParams(
            max_length=20, seed=11, ignore_eos=True))])
        # continuous admission: prompts (some longer than the prefill chunk) join a running
        # session, so mixed prefill+decode steps and chunk steps cross the ring
        from distributed_llm_inferencing_amd.worker.service import PipelineService
        svc = PipelineService(eng, name="pp")
        futs = [svc.submit(p, SamplingParams(max_length=56, do_sample=False, ignore_eos=True))
                for p in PROMPTS[:3]]
        import time
        t0 = time.monotonic()
        while eng.head.stats.decode_steps < 3 and time.monotonic() - t0 < 60:
            time.sleep(0.005)             # the first prompts are decoding
        futs += [svc.submit(p, SamplingParams(max_length=56, do_sample=False, ignore_eos=True))
                 for p in LONG + PROMPTS[3:] + PROMPTS * world]
        res.append([f.result(timeout=200).all_ids for f in futs])
        svc.close()
        res.append(eng.vocab_parallel)
        res.append(eng.head.sched.num_mixed)
        res.append(eng.channel.ipc.stats())
        eng.shutdown()
        q.put(res)
    else:
        eng.serve()
    dist.barrier()
    eng.channel.close()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,vp,mixed,chunk,schedule", [
    (2, "0", "1", 16384, "piped"), (3, "0", "1", 16, "piped"), (2, "1", "0", 16384, "piped"),
    (4, "auto", "1", 16, "piped"), (8, "auto", "1", 16, "piped"), (8, "0", "0", 16384, "piped"),
    # the grouped schedule of the torch / RCCL data plane (serve_session + the head's one
    # grouped exchange per tick), through the same tag-blind FIFO model
    (2, "0", "1", 16384, "grouped"), (3, "1", "1", 16, "grouped"),
    (4, "auto", "1", 16, "grouped"), (8, "auto", "0", 16384, "grouped"),
    (8, "0", "1", 16, "grouped"),
    # every ring size up to a full node: odd sizes, the vocab-parallel head at 5-7 ranks
    (5, "auto", "1", 16, "piped"), (6, "0", "1", 16384, "grouped"), (7, "auto", "0", 16, "piped"),
    (5, "0", "0", 16, "grouped"), (6, "auto", "1", 16, "piped"), (7, "1", "1", 16384, "grouped")])
def test_pipeline_over_fifo_mailboxes_matches_single_stage(world, vp, mixed, chunk, schedule):
    (res,) = _spawn(_pp_worker, world, vp, mixed, chunk, schedule)
    eng = LLMEngine("llama-tiny", device="cpu", dtype=torch.float32, max_batch=8,
                    max_model_len=64, num_blocks=64)
    assert res[0] == [o.all_ids for o in eng.generate(PROMPTS, SamplingParams(
        max_length=20, do_sample=False, ignore_eos=True))]
    assert res[1] == [o.all_ids for o in eng.generate(PROMPTS, SamplingParams(
        max_length=20, seed=11, ignore_eos=True))]
    ref = [o.all_ids for o in eng.generate(PROMPTS[:3] + LONG + PROMPTS[3:] + PROMPTS * world,
                                           SamplingParams(
        max_length=56, do_sample=False, ignore_eos=True))]
    assert res[2] == ref
    assert res[3] == (vp == "1" or (vp == "auto" and world >= 4))
    if mixed == "1":
        assert res[4] > 0                     # mixed steps crossed the ring
    assert res[5]["sends"] > 0 and res[5]["recvs"] > 0


# ------------------------------------------------------------------------------ experts
def _ep_worker(rank, world, port, q, model, shard_dir):
    _env(rank, world, port, DLI_EP_COMM="ipc")
    import torch.distributed as dist
    from distributed_llm_inferencing_amd.parallel.expert import ExpertParallelEngine
    eng = ExpertParallelEngine(model, "cpu", max_batch=8, max_model_len=64, num_blocks=64,
                               dtype=torch.float32, model_dir=shard_dir)
    assert eng.moe.ep is not None
    mine = PROMPTS[rank::world] if rank == 0 else PROMPTS[rank::world][:1]
    sp = SamplingParams(max_length=18, do_sample=False, ignore_eos=True)
    out = [o.all_ids for o in eng.generate(mine, sp)]
    q.put((rank, mine, out, eng.moe.rows_sent, eng.moe.rows_routed, eng.moe.exchanges,
           eng.lockstep_syncs, eng.steps, eng.engine.lookahead))
    dist.barrier()
    eng.moe.close()
    dist.destroy_process_group()


@pytest.mark.parametrize("model,world,from_shards", [("mixtral-tiny", 2, False),
                                                     ("mixtral-tiny", 4, True),
                                                     ("mixtral-tiny8e", 8, False)])
def test_expert_parallel_over_fifo_mailboxes_matches_dense(tmp_path, model, world, from_shards):
    """DP attention + EP experts with the mailbox all-to-all (counts on the device, only
    routed rows on the wire) == one process with all experts, token for token; ranks serve
    different, unequal request sets (idle forwards join every exchange); one lockstep sync
    per step; with ``from_shards`` every rank reads only its experts' rows of the exported
    files."""
    from distributed_llm_inferencing_amd.models import get_config
    shard_dir = None
    if from_shards:
        from distributed_llm_inferencing_amd.shard.writer import export_shards
        paths = export_shards(model, 2, str(tmp_path / "sh"), dtype=torch.float32,
                              log=lambda *a: None)
        shard_dir = str(paths[0].parent)
    res = _spawn(_ep_worker, world, model, shard_dir, n_results=world)
    eng = LLMEngine(model, device="cpu", dtype=torch.float32, max_batch=8, max_model_len=64,
                    num_blocks=64)
    sp = SamplingParams(max_length=18, do_sample=False, ignore_eos=True)
    L = get_config(model).num_layers
    for rank, mine, out, sent, routed, exch, syncs, steps, la in res:
        assert out == [o.all_ids for o in eng.generate(mine, sp)], rank
        assert exch == steps * L and la
        assert syncs == steps + 1                    # the one lockstep exchange per step
        assert sent <= routed                        # no padding rows cross ranks


def _ep_cap_worker(rank, world, port, q):
    """Rank 1 receives its prompts while rank 0 is already decoding: it must admit them in
    chunks of at most max_batch tokens (peers keep their graph-sized steps) and still
    produce the dense model's tokens."""
    _env(rank, world, port, DLI_EP_COMM="ipc")
    import torch.distributed as dist
    from distributed_llm_inferencing_amd.parallel.expert import ExpertParallelEngine
    eng = ExpertParallelEngine("mixtral-tiny", "cpu", max_batch=8, max_model_len=96,
                               num_blocks=64, dtype=torch.float32)
    sp = SamplingParams(max_length=40, do_sample=False, ignore_eos=True)
    early = PROMPTS[:3] if rank == 0 else []
    late = [[(7 * i + j) % 50 + 3 for j in range(20)] for i in range(3)] if rank == 1 else []
    rids = [eng.engine.add_request(p, sp) for p in early]
    outs, steps, big = {}, 0, 0
    while True:
        if steps == 4:
            rids += [eng.engine.add_request(p, sp) for p in late]
        o, more = eng.step()
        outs.update({x.request_id: x.all_ids for x in o})
        steps += 1
        if not more and steps > 4:
            break
    q.put((rank, early + late, [outs[r] for r in rids], eng.capped_steps))
    dist.barrier()
    eng.moe.close()
    dist.destroy_process_group()


def test_expert_parallel_caps_prefill_while_peers_decode():
    res = _spawn(_ep_cap_worker, 2, n_results=2)
    eng = LLMEngine("mixtral-tiny", device="cpu", dtype=torch.float32, max_batch=8,
                    max_model_len=96, num_blocks=64)
    sp = SamplingParams(max_length=40, do_sample=False, ignore_eos=True)
    for rank, prompts, out, capped in res:
        assert out == [o.all_ids for o in eng.generate(prompts, sp)], rank
        if rank == 1:
            assert capped >= 3          # 60 prompt tokens admitted 8 at a time
        else:
            assert capped == 0


# ------------------------------------------------------------------------------ hardening
def _ep_overflow_worker(rank, world, port, q):
    """Rank 0 'replays' a decode graph of bucket 8 holding 5 live rows (every row of the
    bucket is routed), rank 1 is idle (an eager forward of zero rows): rank 1 must reserve a
    region for rank 0's whole bucket, not for its 5 announced tokens."""
    _env(rank, world, port, DLI_EP_COMM="ipc")
    import torch.distributed as dist
    from distributed_llm_inferencing_amd.parallel.expert import ExpertParallelEngine
    eng = ExpertParallelEngine("mixtral-tiny", "cpu", max_batch=8, max_model_len=64,
                               num_blocks=64, dtype=torch.float32)
    moe = eng.moe
    D = eng.cfg.hidden_size
    lp = eng.engine.model.layers[0]
    torch.manual_seed(3)
    h = torch.randn(8, D)
    out = {}
    try:
        if rank == 0:
            # graph replay: the forward runs the padded bucket of 8 rows (a replay performs no
            # host-side check; the lockstep exchange told the peers 5 tokens)
            moe.begin_step([8, 0])
            moe.static = True
            y = moe(h, lp, 0)
            moe.static = False
            moe.begin_step([8, 0])           # the same rows, eagerly, as a reference
            ref = moe(h, lp, 0)
            out["equal"] = bool(torch.allclose(y, ref))
        else:
            moe.begin_step([5, 0])
            moe(h[:0], lp, 0)
            moe.begin_step([8, 0])
            moe(h[:0], lp, 0)
        out["ok"] = True
    except Exception as e:  # noqa: BLE001
        out["ok"] = f"{type(e).__name__}: {e}"
    q.put((rank, out))
    dist.barrier()
    moe.close()
    dist.destroy_process_group()


def test_expert_receive_region_covers_a_replayed_bucket():
    res = dict(_spawn(_ep_overflow_worker, 2, n_results=2))
    assert res[0]["ok"] is True and res[1]["ok"] is True, res
    assert res[0]["equal"]


def _seq_worker(rank, world, port, q):
    _env(rank, world, port)
    import torch.distributed as dist
    dist.init_process_group("gloo")
    from distributed_llm_inferencing_amd.parallel.fifo import (FifoMismatch,
                                                               ShmMailboxTransport, mailbox_caps)
    ep = ShmMailboxTransport(world, rank, mailbox_caps(world, 4096, 4096),
                             f"/dli_fifo_s_{port}", timeout_s=20)
    dist.barrier()
    ep.connect()
    dist.barrier()
    out = {}
    x = torch.arange(16, dtype=torch.int32)
    buf = torch.empty(16, dtype=torch.int32)
    if rank == 0:
        ep.exchange([(x, 1)], [])
        ep.debug_bump_seq(1)                 # the next message carries a wrong sequence
        ep.exchange([(x, 1)], [])
    else:
        ep.exchange([], [(buf, 0)])
        out["first"] = bool(torch.equal(buf, x))
        try:
            ep.exchange([], [(buf, 0)])
            out["second"] = None
        except FifoMismatch as e:
            out["second"] = str(e)
        out["err"] = ep.error()
    q.put((rank, out))
    dist.barrier()
    ep.close()
    dist.destroy_process_group()


def test_mailbox_sequence_check_flags_a_bad_message():
    """Every message carries its edge sequence number (ipc.cpp header); a receiver that
    finds the wrong one (stale / lost / duplicated message) raises instead of delivering."""
    res = dict(_spawn(_seq_worker, 2, n_results=2))
    assert res[1]["first"]
    assert "sequence" in res[1]["second"]
    assert res[1]["err"] & 2


def _resolve_worker(rank, world, port, q):
    _env(rank, world, port)
    import torch.distributed as dist
    dist.init_process_group("gloo")
    from distributed_llm_inferencing_amd.parallel.transport import resolve_comm
    g = dist.new_group(backend="gloo")
    out = {"gpu": resolve_comm("auto", torch.device("cuda", 0), g),
           "cpu": resolve_comm("auto", torch.device("cpu"), g),
           "explicit": resolve_comm("torch", torch.device("cuda", 0), g)}
    q.put((rank, out))
    dist.barrier()
    dist.destroy_process_group()


def test_comm_auto_resolves_to_ipc_for_same_host_gpu_ranks():
    """DLI_PP_COMM / DLI_EP_COMM default "auto": GPU ranks on one host take the device
    mailboxes (the data plane the first 8-GPU run uses); CPU ranks keep torch/gloo."""
    res = dict(_spawn(_resolve_worker, 2, n_results=2))
    for r in (0, 1):
        assert res[r] == {"gpu": "ipc", "cpu": "torch", "explicit": "torch"}
