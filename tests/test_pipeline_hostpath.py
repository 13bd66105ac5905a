"""Pipeline host path at the 8-GPU shape, on CPU: an 8-rank gloo ring whose stages do no
model compute ("null compute": every stage returns a view of a buffer allocated once), with
the real scheduler, metadata packing, shared-memory control ring and data-plane exchange,
512-row microbatches and the vocab-parallel head of the N >= 4 default. It bounds

* the head's host time per tick (everything the head does between ticks except waiting
  for the transport): <= 0.5 ms per decode tick, so the head's host keeps up with the
  ~1.2 ms decode tick of a 4-layer Llama-3-8B stage at 512 rows (and <= 1 ms averaged over
  every tick, prefill and finishing ticks included);
* tensor allocations in the transport / pipeline loops: zero per steady-state tick on
  every rank (counted with a TorchDispatchMode over all aten factory / copy ops).

The control plane must be the shared-memory ring (all ranks on one host)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

ALLOC_OPS = ("empty", "zeros", "ones", "full", "clone", "_to_copy", "new_empty", "new_zeros",
             "cat", "stack", "empty_like", "zeros_like", "randn", "rand", "arange")


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _patch_null_compute():
    """Stage compute / candidates / sampling replaced by views of preallocated buffers.
    Candidates are 8 per rank (the requests use top_k 8): the head's host work does not
    depend on the width, but 64-wide candidates from 7 ranks put ~2 MB of loopback TCP
    per tick on this 8-core container (RCCL over xGMI on the GPU node)."""
    from distributed_llm_inferencing_amd.parallel import pipeline as P
    P.CAND = 8

    def compute(self, meta, data):
        if meta.num_seqs == 0:
            return None
        bufs = getattr(self, "_null", None)
        if bufs is None:
            D = self.cfg.hidden_size
            self._null = bufs = (torch.zeros(self.max_tokens, D, dtype=torch.float32),
                                 torch.full((self.max_batch,), 7, dtype=torch.int32),
                                 torch.zeros(self.max_batch, D, dtype=torch.float32))
        if self.is_last:
            if self.vocab_parallel:
                return bufs[2][:meta.num_seqs]
            return bufs[1][:meta.num_seqs]
        return bufs[0][:meta.num_tokens]

    def candidates(self, hf):
        c = getattr(self, "_null_c", None)
        if c is None:
            c = torch.zeros(self.max_batch, 2 * P.CAND, dtype=torch.int32)
            c[:, P.CAND:] = torch.arange(P.CAND, dtype=torch.int32) + 3
            self._null_c = c
        return c[:hf.shape[0]]

    def sample_candidates(self, meta, packed):
        t = getattr(self, "_null_t", None)
        if t is None:
            self._null_t = t = torch.full((self.max_batch,), 9, dtype=torch.int32)
        return t[:meta.num_seqs]

    P.StageWorker.compute = compute
    P.StageWorker.candidates = candidates
    P.StageWorker.sample_candidates = sample_candidates


class _AllocCounter(torch.utils._python_dispatch.TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.counts = {}

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        name = func.__name__.split(".")[0]
        if name in ALLOC_OPS:
            self.counts[name] = self.counts.get(name, 0) + 1
        return func(*args, **(kwargs or {}))


def _worker(rank, world, port, q, batch, n_req):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank), DLI_PP_VOCAB_PARALLEL="auto",
                      DLI_PP_TICK_LOG="1")
    torch.set_num_threads(1)
    import torch.distributed as dist
    from distributed_llm_inferencing_amd.engine import SamplingParams
    from distributed_llm_inferencing_amd.parallel import pipeline as P
    _patch_null_compute()
    # 8 layers (one per stage), narrow hidden state: the data plane's CPU/TCP copies are not
    # what this test measures (on the GPU node they are RCCL transfers over xGMI)
    from dataclasses import replace
    from distributed_llm_inferencing_amd.models.configs import get_config, register
    register(replace(get_config("llama-tiny8"), name="llama-null8", hidden_size=64,
                     num_heads=1, num_kv_heads=1, head_dim=64, intermediate_size=128))
    eng = P.DistributedPipelineEngine("llama-null8", "cpu", max_batch=batch, max_model_len=64,
                                      num_blocks=24576, dtype=torch.float32,
                                      max_prefill_tokens=batch * 8)
    sp = SamplingParams(max_length=40, temperature=0.8, top_k=8, top_p=0.95, ignore_eos=True)
    rng = np.random.default_rng(0)
    prompts = [rng.integers(3, 1000, size=8).tolist() for _ in range(n_req)]
    if rank == 0:
        eng.generate(prompts[:batch], sp)               # warm session (numpy / ctypes paths)
        eng.head.host_s, eng.head.ticks = 0.0, 0
        eng.head.host_by_kind = {k: [0.0, 0] for k in eng.head.host_by_kind}
        eng.head.tick_log = []
        outs = eng.generate(prompts, sp)                # timed session
        dec = sorted(t[1] for t in eng.head.tick_log if t[0] == 2)
        dec_cpu = sorted(t[7] for t in eng.head.tick_log if t[0] == 2)
        dec_ph = np.array([t[2:7] for t in eng.head.tick_log if t[0] == 2])
        ph_p50 = dict(zip(("finish", "schedule", "ctrl", "head_ops", "compute"),
                          np.round(1e3 * np.median(dec_ph, axis=0), 4).tolist()))
        ticks, host_s = eng.head.ticks, eng.head.host_s
        dec_s, dec_n = eng.head.host_by_kind[2]
        phases = dict(eng.head.phase_s)
        # counted session: allocations from the first decode tick on
        for p in prompts[:2 * batch]:
            eng.add_request(p, sp)
        counter = _AllocCounter()
        orig = eng.head.sched.schedule
        state = {"on": False}

        def sched(mb, *a, **kw):
            m = orig(mb, *a, **kw)
            if m is not None and m.kind == 2 and not state["on"]:
                state["on"] = True
                counter.__enter__()
            return m
        eng.head.sched.schedule = sched
        eng.head.run_session()
        if state["on"]:
            counter.__exit__(None, None, None)
        eng.shutdown()
        res = dict(rank=0, ticks=ticks, host_ms=1e3 * host_s / max(1, ticks),
                   decode_ticks=dec_n, decode_host_ms=1e3 * dec_s / max(1, dec_n),
                   decode_host_ms_p50=1e3 * dec[len(dec) // 2],
                   decode_cpu_ms_p50=1e3 * dec_cpu[len(dec_cpu) // 2],
                   decode_cpu_ms=1e3 * sum(dec_cpu) / max(1, len(dec_cpu)),
                   decode_phase_ms_p50=ph_p50,
                   allocs=counter.counts, n_out=len(outs),
                   toks=sum(len(o.output_ids) for o in outs), ctrl=eng.channel.ctrl_kind,
                   vp=eng.vocab_parallel, M=eng.microbatches,
                   phases={k: round(1e3 * v / max(1, ticks), 4) for k, v in phases.items()})
    else:
        from distributed_llm_inferencing_amd.engine.batch import DECODE
        bufs = P._StageBuffers(eng.stage, eng.channel)
        P.serve_session(eng.stage, eng.channel, bufs)  # warm session
        P.serve_session(eng.stage, eng.channel, bufs)  # timed session
        counter = _AllocCounter()
        orig_unpack = P.StepMeta.unpack
        state = {"on": False}

        def unpack(h, p):
            m = orig_unpack(h, p)
            if m.kind == DECODE and not state["on"]:
                state["on"] = True
                counter.__enter__()
            return m
        P.StepMeta.unpack = staticmethod(unpack)
        P.serve_session(eng.stage, eng.channel, bufs)
        if state["on"]:
            counter.__exit__(None, None, None)
        P.serve_session(eng.stage, eng.channel, bufs)  # SHUTDOWN
        res = dict(rank=rank, allocs=counter.counts, ctrl=eng.channel.ctrl_kind)
    q.put(res)
    dist.barrier()
    eng.channel.close()
    dist.destroy_process_group()


def _run_ring(world, batch):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    M = world + 3                          # vocab-parallel head at N = 8
    n_req = batch * M
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, batch, n_req))
             for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        r = q.get(timeout=600)
        res[r["rank"]] = r
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    head = res[0]
    print("head:", head)
    assert head["ctrl"] == "shm" and all(r["ctrl"] == "shm" for r in res.values())
    assert head["vp"] and head["M"] == M
    assert head["n_out"] == n_req and head["toks"] == n_req * (40 - 8)
    assert head["ticks"] > 300
    for r, v in sorted(res.items()):
        assert v["allocs"] == {}, (r, v["allocs"])
    assert head["decode_ticks"] > 300
    return head


def _fast_enough(head):
    # steady state (decode ticks: ~1.2 ms of GPU work each at the 8-GPU shape) and overall
    # (prefill ticks hide behind ~20 ms of prefill GPU work; finishing ticks are rare)
    # (median: robust to OS scheduling noise on a shared CI host; the means are bounded too)
    return (head["decode_host_ms_p50"] <= 0.5 and head["decode_host_ms"] <= 0.75
            and head["host_ms"] <= 1.0)


def test_null_compute_ring_host_path_n8():
    """8 ranks on an 8-CPU host: a loaded host (a build, another test process) inflates the
    host times of one run, so a run over the bounds is repeated once and the second run
    must meet them (the functional checks hold on both)."""
    head = _run_ring(8, 512)
    if not _fast_enough(head):
        head = _run_ring(8, 512)
    if not _fast_enough(head) and os.environ.get("PYTEST_XDIST_WORKER"):
        # 8 ranks beside other xdist workers on 8 CPUs: the functional checks passed, the
        # host-time bounds only mean something on an unloaded host (the serial run checks them)
        pytest.skip(f"host-time bounds need an unloaded host (pytest -n): {head}")
    assert _fast_enough(head), head
