"""The device mailbox data plane (csrc/runtime/ipc.cpp) hardened for the first 8-GPU run:
uncached mailboxes, per-message sequence checks, sticky failure, and a ring that notices a
dead stage in well under the wait budget (the reference has no data
plane at all: master/dashboard/views.py:318-355, worker/app.py:332-372).

All ranks share cuda:0 (gloo for the control group: RCCL refuses two ranks on one GPU)."""
import os
import socket
import time

import pytest
import torch
import torch.multiprocessing as mp

from distributed_llm_inferencing_amd.engine import SamplingParams

pytestmark = pytest.mark.gpu
PROMPTS = [[5, 6, 7, 8], [9, 10, 11], [1, 2, 3, 4, 5, 6, 7], [100, 200], [7] * 9, [3, 4]]
GREEDY = SamplingParams(max_length=40, do_sample=False, ignore_eos=True)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _env(rank, world, port, **extra):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank), DLI_DIST_BACKEND="gloo",
                      DLI_SAME_DEVICE="1", DLI_GEMM_AUTOTUNE="0", **extra)
    os.environ.pop("DLI_PP_COMM", None)
    os.environ.pop("DLI_EP_COMM", None)


def _spawn(target, world, *args, n_results=None, timeout=240, ok_codes=(0,)):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, q) + args) for r in range(world)]
    for p in procs:
        p.start()
    try:
        res = [q.get(timeout=timeout) for _ in range(n_results or world)]
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    codes = [p.exitcode for p in procs]
    assert all(c in ok_codes for c in codes), codes
    return res


# ------------------------------------------------------------------------------ endpoint
def _ep_worker(rank, world, port, q):
    _env(rank, world, port)
    import torch.distributed as dist
    dist.init_process_group("gloo")
    torch.cuda.set_device(0)
    from distributed_llm_inferencing_amd.parallel.fifo import mailbox_caps
    from distributed_llm_inferencing_amd.parallel.transport import ipc_selftest
    from distributed_llm_inferencing_amd.runtime import IpcEndpoint
    ep = IpcEndpoint(world, rank, mailbox_caps(world, 1 << 20, 1 << 16))
    hs = [None] * world
    dist.all_gather_object(hs, ep.handles())
    dist.barrier()
    ep.connect(hs)
    dist.barrier()
    out = {"kind": ep.mem_kind, "selftest": ipc_selftest(ep, dist.group.WORLD)}
    st = torch.cuda.current_stream().cuda_stream
    dev = torch.device("cuda", 0)
    x = (torch.arange(4096, dtype=torch.float32, device=dev) + 7 * rank).to(torch.bfloat16)
    odd = torch.arange(13, dtype=torch.int32, device=dev)[1:] + rank   # 4-B aligned only
    buf = torch.empty_like(x)
    obuf = torch.empty_like(odd)
    nxt, prv = (rank + 1) % world, (rank - 1) % world
    for _ in range(3):          # FIFO round trips, data checked (one message per edge in
        ep.exchange([(x, nxt)], [(buf, prv)], st)           # flight: the mailbox holds one)
        ep.exchange([(odd, nxt)], [(obuf, prv)], st)
    torch.cuda.synchronize()
    want = (torch.arange(4096, dtype=torch.float32, device=dev) + 7 * prv).to(torch.bfloat16)
    out["data"] = bool(torch.equal(buf, want)
                       and torch.equal(obuf, torch.arange(13, dtype=torch.int32,
                                                          device=dev)[1:] + prv))
    out["err0"] = ep.error()
    dist.barrier()
    # rank 0 stamps a wrong sequence number on its next message to rank 1: rank 1 must flag
    # it (and never deliver it silently), then its queue drains fast (sticky failure)
    ep.set_wait(5.0)
    if rank == 0:
        ep.debug_bump_seq(1, st)
    t0 = time.monotonic()
    try:
        ep.exchange([(x, nxt)], [(buf, prv)], st)
        ep.exchange([(x, nxt)], [(buf, prv)], st)
        torch.cuda.synchronize()
    except Exception as e:  # noqa: BLE001
        out["raise"] = str(e)
    out["drain_s"] = time.monotonic() - t0
    out["err1"] = ep.error()
    q.put((rank, out))
    dist.barrier()
    ep.close()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_ipc_mailboxes_uncached_sequenced_and_sticky(gpu):
    res = dict(_spawn(_ep_worker, 2))
    for r in (0, 1):
        assert res[r]["kind"] == "uncached", res[r]
        assert res[r]["selftest"] and res[r]["data"] and res[r]["err0"] == 0, res[r]
    assert res[1]["err1"] & 2, res[1]                 # the corrupted message was flagged
    # the flagged rank stops signalling; its peer's next wait runs out of budget (5 s) or
    # the queue is released, never a hang
    # (its first message still landed; its next waits run out of budget: bit 0, and the
    # stale mailbox it then reads is flagged too: bit 1)
    assert res[0]["err1"] in (0, 1, 3), res[0]
    assert res[1]["drain_s"] < 10 and res[0]["drain_s"] < 10, res


# ------------------------------------------------------------------------------ pipeline
def _pp_worker(rank, world, port, q, corrupt):
    _env(rank, world, port, DLI_PP_VOCAB_PARALLEL="0", DLI_IPC_WAIT_S="5",
         DLI_FAULT="pipeline.stage:exit_after:150" if (rank == 1 and not corrupt) else "")
    import torch.distributed as dist
    from distributed_llm_inferencing_amd.parallel.pipeline import DistributedPipelineEngine
    eng = DistributedPipelineEngine("llama-tiny", "cuda", max_batch=8, max_model_len=128,
                                    num_blocks=256)
    eng.warmup()
    out = {"comm": eng.channel.comm, "kind": getattr(eng.channel.ipc, "mem_kind", None)}
    if rank != 0:
        try:
            eng.serve()
        except BaseException as e:  # noqa: BLE001 — the head died / the plane failed
            out["stage_error"] = f"{type(e).__name__}: {e}"
        q.put((rank, out))
        return
    ok = [o.all_ids for o in eng.generate(PROMPTS[:2], GREEDY)]
    out["first"] = len(ok)
    if corrupt:
        eng.channel.ipc.debug_bump_seq(1, torch.cuda.current_stream().cuda_stream)
    t0 = time.monotonic()
    try:
        eng.generate(PROMPTS * 4, SamplingParams(max_length=120, do_sample=False,
                                                 ignore_eos=True))
        out["error"] = None
    except BaseException as e:  # noqa: BLE001
        out["error"] = f"{type(e).__name__}: {e}"
    out["fail_s"] = time.monotonic() - t0
    out["dead"] = eng.channel.dead_peer
    eng.channel.abort_data_plane()
    out["drained"] = eng.channel.drain(timeout_s=10.0)
    q.put((rank, out))
    q.close()
    q.join_thread()
    os._exit(0)                           # the stage side may be gone: no goodbye


@pytest.mark.timeout(300)
def test_pipeline_defaults_to_ipc_and_fails_fast_when_a_stage_dies(gpu):
    """PP N=2 on one GPU with NO data-plane env override: the channel resolves to the IPC
    mailboxes (uncached). Stage 1 hard-exits mid-session (injected fault): the head's
    watchdog notices the dead pid, aborts the mailboxes (every queued wait returns), and the
    session raises within seconds, not after a wait budget; the head's stream drains."""
    res = dict(_spawn(_pp_worker, 2, False, n_results=1, ok_codes=(0, 17)))
    head = res[0]
    assert head["comm"] == "ipc" and head["kind"] == "uncached", head
    assert head["first"] == 2
    assert head["error"] is not None and "stage 1" in head["error"], head
    assert head["fail_s"] < 5.0, head
    assert head["drained"], head


@pytest.mark.timeout(300)
def test_pipeline_stale_message_surfaces_as_error_not_tokens(gpu):
    """The head corrupts the sequence number of its next activation message to stage 1:
    stage 1 flags it and stops signalling, and the head's session raises (DataPlaneError /
    PeerDied) instead of returning tokens computed from a stale mailbox."""
    res = dict(_spawn(_pp_worker, 2, True, n_results=2, ok_codes=(0,)))
    head, stage = res[0], res[1]
    assert head["error"] is not None, head
    assert "IPC data plane error" in head["error"] or "stage" in head["error"], head
    assert stage.get("stage_error") and "sequence" in stage["stage_error"], stage
    assert head["fail_s"] < 15.0, head
