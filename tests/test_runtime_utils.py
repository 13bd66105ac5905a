"""C++ runtime (block allocator, safetensors loader), fault injection, tracing, and engine
edge cases (preemption, deadlines, HF max_length semantics) on CPU."""
import json
import os

import numpy as np
import pytest
import torch

from distributed_llm_inferencing_amd.engine import SamplingParams
from distributed_llm_inferencing_amd.engine.llm_engine import LLMEngine
from distributed_llm_inferencing_amd.runtime import BlockManager, SafetensorsFile
from distributed_llm_inferencing_amd.utils import faults
from distributed_llm_inferencing_amd.utils.tracing import SpanLog, StepTimer, trace_range


def test_block_manager_alloc_free_tables():
    bm = BlockManager(8, 16)
    assert bm.num_free == 8
    assert bm.ensure(1, 20)                     # 2 blocks
    assert bm.ensure(1, 32) and bm.num_free == 6
    assert bm.ensure(1, 33) and bm.num_free == 5
    assert bm.blocks_needed(2, 100) == 7
    assert not bm.ensure(2, 100)                # all-or-nothing
    assert bm.num_free == 5 and bm.table(2) == []
    t = bm.table(1)
    assert len(t) == 3 and len(set(t)) == 3
    tabs = bm.fill_tables([1, 2], 4)
    assert tabs.shape == (2, 4) and tabs[0, :3].tolist() == t and tabs[1].tolist() == [0] * 4
    slots = bm.slot_mapping([1], [15], [3])
    assert slots.tolist() == [t[0] * 16 + 15, t[1] * 16, t[1] * 16 + 1]
    with pytest.raises(RuntimeError):
        bm.fill_tables([1], 2)                  # wider than max_blocks
    assert bm.free(1) == 3 and bm.num_free == 8


def test_safetensors_cpp_loader_roundtrip(tmp_path):
    from safetensors.torch import save_file
    ts = {"a": torch.randn(7, 9).to(torch.bfloat16), "b.c": torch.arange(11, dtype=torch.int32),
          "d": torch.randn(3, 4, 5)}
    p = tmp_path / "x.safetensors"
    save_file(ts, str(p), metadata={"k": "v"})
    f = SafetensorsFile(str(p))
    assert set(f.keys()) == set(ts)
    out = f.load()
    for k in ts:
        assert out[k].dtype == ts[k].dtype and torch.equal(out[k], ts[k])
    part = f.load(["b.c"])
    assert list(part) == ["b.c"]
    f.close()
    with pytest.raises(IOError):
        SafetensorsFile(str(tmp_path / "missing.safetensors"))


def test_fault_injection_rules():
    faults.reload("worker.inference:error,transport.exchange:error:3,x.y:delay:1")
    with pytest.raises(faults.InjectedFault):
        faults.check("worker.inference")
    faults.check("transport.exchange", tick=2)           # other ticks pass
    with pytest.raises(faults.InjectedFault):
        faults.check("transport.exchange", tick=3)
    faults.check("x.y")
    faults.check("unrelated.site")
    assert faults.stats()["worker.inference:error"] == 1
    faults.reload("")
    assert not faults.active()


def test_worker_fault_injection_http(tmp_path, monkeypatch):
    from distributed_llm_inferencing_amd.config import Settings
    from distributed_llm_inferencing_amd.worker.server import create_worker_app
    s = Settings()
    s.model_cache_dir = str(tmp_path)
    c = create_worker_app(s, device="cpu", engine_kwargs=dict(max_batch=4, max_model_len=64,
                                                              num_blocks=32)).test_client()
    faults.reload("worker.health:error,worker.inference:error")
    try:
        assert c.get("/health").status_code == 503
        r = c.post("/inference", json={"model_name": "llama-tiny", "prompt": "hi"})
        assert r.status_code == 500 and "injected fault" in r.get_json()["message"]
    finally:
        faults.reload("")
    assert c.get("/health").status_code == 200


def test_tracing_spans_and_timer(tmp_path, monkeypatch):
    log = tmp_path / "req.jsonl"
    monkeypatch.setenv("DLI_REQUEST_LOG", str(log))
    eng = LLMEngine("llama-tiny", device="cpu", max_batch=4, max_model_len=64, num_blocks=32)
    with trace_range("noop"):
        eng.generate([[1, 2, 3]], SamplingParams(max_length=8))
    rec = [json.loads(x) for x in log.read_text().splitlines()]
    assert rec[0]["output_tokens"] == 5 and rec[0]["ttft_s"] is not None
    snap = eng.timer.snapshot()
    assert {"schedule", "run_prefill", "run_decode", "sync", "update"} <= set(snap)
    t = StepTimer()
    with t.phase("a"):
        pass
    assert t.snapshot()["a"]["calls"] == 1


def test_max_length_semantics_and_budget():
    eng = LLMEngine("llama-tiny", device="cpu", max_batch=4, max_model_len=64, num_blocks=32)
    outs = eng.generate([[5] * 10, [5] * 3], SamplingParams(max_length=10))
    assert outs[0].output_ids == [] and outs[0].finish_reason == "length"   # prompt >= max_length
    assert len(outs[1].all_ids) == 10
    o = eng.generate([[5] * 3], SamplingParams(max_new_tokens=4))[0]
    assert len(o.output_ids) == 4


def test_deadline_enforced_per_step():
    eng = LLMEngine("llama-tiny", device="cpu", max_batch=4, max_model_len=256, num_blocks=64)
    o = eng.generate([[5] * 3], SamplingParams(max_length=200, timeout_s=0.0))[0]
    assert o.finish_reason == "timeout" and len(o.output_ids) < 197


def test_preemption_under_kv_pressure_keeps_outputs():
    """8 blocks of 16 tokens cannot hold 4 sequences of 48 tokens at once: the scheduler
    preempts + recomputes, and greedy outputs equal an unconstrained run."""
    prompts = [[i + 3] * 8 for i in range(4)]
    sp = SamplingParams(max_length=48, do_sample=False, ignore_eos=True)
    big = LLMEngine("llama-tiny", device="cpu", dtype=torch.float32, max_batch=4,
                    max_model_len=64, num_blocks=64).generate(prompts, sp)
    small_eng = LLMEngine("llama-tiny", device="cpu", dtype=torch.float32, max_batch=4,
                          max_model_len=64, num_blocks=8)
    small = small_eng.generate(prompts, sp)
    assert [o.all_ids for o in small] == [o.all_ids for o in big]
    assert small_eng.bm.num_free == 8


def test_runtime_host_asan_selftest():
    """The C++ runtime under host AddressSanitizer: allocator stress + safetensors parser
    fuzz (truncated headers, bad lengths, out-of-range offsets)."""
    import shutil
    import subprocess
    from distributed_llm_inferencing_amd import build
    if shutil.which("hipcc") is None and not os.path.exists("/opt/rocm/bin/hipcc"):
        pytest.skip("hipcc not available")
    exe = build.build_asan_selftest(verbose=False)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1")
    r = subprocess.run([str(exe)], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "runtime_selftest: OK" in r.stdout


def test_stale_native_library_is_rebuilt_or_refused(tmp_path, monkeypatch):
    """A library whose source-digest stamp does not match the tree is rebuilt when hipcc is
    present and refused (not loaded) when it is not; a current one is left alone."""
    from distributed_llm_inferencing_amd import build as B
    from distributed_llm_inferencing_amd.ops._native import ensure_current
    lib = tmp_path / "libfake.so"
    lib.write_bytes(b"\x7fELF")
    B.stamp_path(lib).write_text("0" * 40)                       # built from other sources
    assert not B.is_current("kernels", lib)

    def no_hipcc():
        raise RuntimeError("hipcc not found")
    monkeypatch.setattr(B, "_hipcc", no_hipcc)
    with pytest.raises(RuntimeError, match="stale"):
        ensure_current(lib, "kernels")

    monkeypatch.setattr(B, "_hipcc", lambda: "/opt/rocm/bin/hipcc")
    calls = []

    def fake_build(verbose=False):
        calls.append(1)
        B.stamp_path(lib).write_text(B.source_digest("kernels"))
    monkeypatch.setattr(B, "build", fake_build)
    ensure_current(lib, "kernels")
    assert calls == [1] and B.is_current("kernels", lib)
    ensure_current(lib, "kernels")                                # current: no rebuild
    assert calls == [1]
    # the in-tree libraries are stamped by the real build
    assert B.is_current("kernels", B.LIBDIR / "libdli_kernels.so")
    assert B.is_current("runtime", B.LIBDIR / "libdli_runtime.so")


def test_shm_ring_broadcast_order_backpressure_and_dead_producer():
    import os
    import numpy as np
    from distributed_llm_inferencing_amd.runtime import ShmRing
    name = f"/dli_test_{os.getpid()}"
    r = ShmRing.create(name, 4, 256, 2)
    a, b = ShmRing.open(name, 0), ShmRing.open(name, 1)
    r.unlink()
    for i in range(4):                                            # fills every slot
        r.publish(np.full(i + 1, i, np.int32))
    with pytest.raises(TimeoutError):                             # consumers are behind
        r.publish(np.zeros(1, np.int32), timeout_s=0.2)
    for i in range(4):
        assert a.consume().view(np.int32).tolist() == [i] * (i + 1)
    with pytest.raises(TimeoutError):                             # b still holds slot 0
        r.publish(np.zeros(1, np.int32), timeout_s=0.2)
    for i in range(4):
        assert b.consume().view(np.int32).tolist() == [i] * (i + 1)
    r.publish(np.arange(3, dtype=np.int64))
    assert a.consume().view(np.int64).tolist() == [0, 1, 2]
    with pytest.raises(ValueError):
        r.publish(np.zeros(100, np.int64))                       # larger than a slot
    r.close()
    assert b.consume().view(np.int64).tolist() == [0, 1, 2]      # drained, then closed
    with pytest.raises(EOFError):
        b.consume(timeout_s=1.0)
    for x in (a, b, r):
        x.destroy()


def _open_ring_and_exit(name):
    from distributed_llm_inferencing_amd.runtime import ShmRing
    ShmRing.open(name, 0)
    os._exit(0)


def test_shm_ring_reports_an_unreaped_consumer_as_dead():
    """A stage that exited while its launcher is blocked elsewhere stays a zombie (kill(pid,
    0) still succeeds): the ring's liveness check reads its state and reports it dead."""
    import multiprocessing as mproc
    import time
    from distributed_llm_inferencing_amd.runtime import ShmRing
    name = f"/dli_ztest_{os.getpid()}"
    r = ShmRing.create(name, 4, 256, 1)
    assert r.dead() == -1                          # never opened: counts as alive
    p = mproc.get_context("fork").Process(target=_open_ring_and_exit, args=(name,))
    p.start()
    t0 = time.monotonic()
    while r.dead() != 0 and time.monotonic() - t0 < 10:
        time.sleep(0.05)
    try:
        assert r.dead() == 0                       # the child is a zombie: not reaped yet
    finally:
        p.join()
        r.unlink()
        r.destroy()


def test_decode_core_matches_python_scheduler():
    """The C++ decode fast path (DecodeCore) builds the same step metadata and applies
    tokens exactly like the numpy path, including finishing rows and preemption."""
    import numpy as np
    from distributed_llm_inferencing_amd.engine.scheduler import Scheduler
    from distributed_llm_inferencing_amd.engine.sequence import SamplingParams
    from distributed_llm_inferencing_amd.runtime import BlockManager

    def run(native):
        s = Scheduler(BlockManager(40, 4), max_seqs_per_mb=16, max_prefill_tokens=64,
                      num_microbatches=2, eos_token_id=2, max_model_len=40,
                      native_decode=native)
        rng = np.random.default_rng(1)
        for i in range(10):
            s.add_request(f"r{i}", rng.integers(3, 90, size=3 + i % 4).tolist(),
                          SamplingParams(max_length=12 + i, seed=i, ignore_eos=i % 2 == 0))
        metas, k = [], 0
        inflight = {}
        while s.has_work() or inflight:
            j = k - 2
            if j in inflight:
                m = inflight.pop(j)
                toks = (np.asarray(m.seq_ids, np.int64) * 7 + k) % 50 + 1   # some are EOS (2)
                s.update(m, toks.astype(np.int32))
            m = s.schedule(k % 2) if s.has_work() else None
            if m is not None:
                h, p = m.pack()
                metas.append((h.tolist(), p.tolist()))
                inflight[k] = m
            k += 1
        return metas, sorted((q.request_id, q.output_ids, q.finish_reason)
                             for q in s.pop_finished())
    m_py, out_py = run(False)
    m_c, out_c = run(True)
    assert out_c == out_py
    assert m_c == m_py


def test_prefill_gemm_plan_is_own_kernel(monkeypatch):
    """Prefill-sized GEMMs plan onto the 8-phase MFMA kernel (tile 22); every plan the
    planner or the autotune can produce is one of our kernels (no library backend left)."""
    from distributed_llm_inferencing_amd.ops import gemm as G
    G.clear_plans()
    for epi in ("none", "silu_mul", "splitk", "f32"):
        p = G.plan(16384, 6144, 4096, epi)
        assert p.backend == "dli" and p.tile == 22 and p.splits == 1, (epi, p)
    # mid-sized steps split K until the grid fills the chip (no split for fused epilogues)
    assert G.plan(1200, 6144, 4096, "splitk") == G.GemmPlan("dli", 22, 2)      # 120 tiles
    assert G.plan(1200, 4096, 4096, "none") == G.GemmPlan("dli", 22, 2)        # 80 tiles
    assert G.plan(1100, 4096, 14336, "splitk") == G.GemmPlan("dli", 22, 2)
    assert G.plan(1024, 4096, 4096, "splitk") == G.GemmPlan("dli", 22, 4)      # 64 tiles
    assert G.plan(1200, 28672, 4096, "silu_mul").splits == 1
    assert all(p.backend == "dli" for p in G.candidate_plans(512, 4096, 4096, "none"))
    # mixed prefill+decode steps of a full batch (512 < M < 1024): 8-phase tiles, and one
    # plan-cache bucket per 128 rows (tuned when serving: StageRunner.autotune_mixed)
    assert G.plan(800, 28672, 4096, "silu_mul") == G.GemmPlan("dli", 22, 1)
    assert G.plan(600, 4096, 14336, "splitk").tile == 22
    assert [G._bucket(m) for m in (512, 513, 640, 641, 1000, 1024, 1025)] == \
        [512, 640, 640, 768, 1024, 1024, 2048]
    G.set_plan(700, 4096, 4096, "splitk", G.GemmPlan("dli", 16, 4))
    assert G.plan(650, 4096, 4096, "splitk") == G.GemmPlan("dli", 16, 4)   # same bucket
    # 256x224 joins the autotune candidates where it lands on whole waves of the chip
    assert not any(p.tile == 26 for p in G.candidate_plans(512, 28672, 4096, "silu_mul"))
    assert any(p.tile == 26 for p in G.candidate_plans(512, 57344, 8192, "silu_mul"))
    # batch 1-2 gate/up: the 16-row SiLU weight stream (tile 29, 8 gate + 8 up rows per
    # workgroup); it competes in the decode autotune up to M = 4 and never outside SiLU
    assert G.plan(1, 28672, 4096, "silu_mul") == G.GemmPlan("dli", 29, 1)
    assert G.plan(2, 28672, 4096, "silu_mul").tile == 29
    assert any(p.tile == 29 for p in G.candidate_plans(4, 28672, 4096, "silu_mul"))
    assert not any(p.tile == 29 for p in G.candidate_plans(1, 4096, 4096, "splitk"))
    assert not any(p.tile == 29 for p in G.candidate_plans(8, 28672, 4096, "silu_mul"))
    G.clear_plans()
    # prefill autotune (StageRunner.autotune_prefill): our 8-phase plan vs our 4-wave plan at
    # the same split
    # (and the persistent 4-wave tile 55 where the plan is unsplit and K an even K-tile count)
    c = G.prefill_candidates(16384, 28672, 4096, "silu_mul")
    t4 = G.PREFILL_4W_TILE
    assert c == [G.GemmPlan("dli", 22, 1), G.GemmPlan("dli", t4, 1), G.GemmPlan("dli", 55, 1)]
    assert G.prefill_candidates(2048, 4096, 4096, "splitk") == \
        [G.GemmPlan("dli", 22, 2), G.GemmPlan("dli", t4, 2)]
    assert G.GemmPlan("dli", 55, 1) not in G.prefill_candidates(16384, 4096, 4160, "none")
    assert all(p.backend == "dli" for p in G.prefill_candidates(4096, 4096, 4096, "bias_gelu"))
    for env in ("DLI_TUNE_PREFILL_LIB", "DLI_GEMM_PREFILL_LIB", "DLI_GEMM_DECODE_LIB"):
        monkeypatch.setenv(env, "1")             # no switch reaches a library backend
    monkeypatch.setenv("DLI_GEMM_BACKEND", "library")
    G.clear_plans()
    assert G.plan(16384, 6144, 4096, "none") == G.GemmPlan("dli", 22, 1)
    assert [p.backend for p in G.prefill_candidates(16384, 6144, 4096, "none")] == ["dli"] * 3
    assert all(p.backend == "dli" for p in G.candidate_plans(512, 4096, 4096, "splitk"))
    G.clear_plans()
    # the 4-wave tiles stay out of the decode autotune (tile 41 cost the step 1.8 %)
    tiles = {p.tile for p in G.candidate_plans(512, 4096, 4096, "none")}
    assert not tiles & {34, 41, 45, 55} and 22 in tiles
    # decode QKV timing pins the candidate for the fused attention path, then restores
    p1, p4 = G.GemmPlan("dli", 30, 1), G.GemmPlan("dli", 32, 4)
    G.set_plan(1, 6144, 4096, "none", p4)
    with G._forced_plan(1, 6144, 4096, p1):
        assert G.plan(1, 6144, 4096, "splitk") == p1 and G.plan(1, 6144, 4096, "none") == p1
    assert G._plan_cache[(1, 6144, 4096, "none")] == p4
    assert (1, 6144, 4096, "splitk") not in G._plan_cache
    with G._forced_plan(1, 6144, 4096, p4):
        assert G.plan(1, 6144, 4096, "splitk") == p4
    G.clear_plans()


def test_slice_experts_releases_other_experts():
    """An EP rank keeps only its experts' storage (a view would pin all of them)."""
    import torch
    from distributed_llm_inferencing_amd.models import weights as W
    t = torch.randn(8, 16, 4)
    s = W.slice_experts("layers.0.w_gu", t, (2, 4))
    assert s.shape[0] == 2 and torch.equal(s, t[2:4])
    assert s.untyped_storage().nbytes() == 2 * 16 * 4 * 4
    assert W.slice_experts("layers.0.attn_norm", t, (2, 4)) is t


def test_build_refuses_scratch_in_asm_mfma_kernels():
    """build.check_scratch: an inline-asm-MFMA kernel (gemm4w) that spills its accumulators
    to scratch fails the build (hipcc pads no hazard after the asm; a rolled bias-GELU
    epilogue did exactly this and returned intermittently wrong tiles); other kernels and a
    zero scratch size pass."""
    from distributed_llm_inferencing_amd import build
    ok = ("gemm.hip:1:1: remark: Function Name: _Z13gemm4w_kernelILi3ELi9EEvPKti\n"
          "gemm.hip:1:1: remark:     ScratchSize [bytes/lane]: 0\n"
          "gemm.hip:1:1: remark: Function Name: _Z9other_kernelv\n"
          "gemm.hip:1:1: remark:     ScratchSize [bytes/lane]: 64\n")
    build.check_scratch(ok, "gemm.hip")
    bad = ok + ("gemm.hip:1:1: remark: Function Name: _Z13gemm4w_kernelILi3ELi8EEvPKti\n"
                "gemm.hip:1:1: remark:     ScratchSize [bytes/lane]: 1040\n")
    with pytest.raises(RuntimeError, match="1040 B/lane"):
        build.check_scratch(bad, "gemm.hip")


def test_gemm_workspace_growth_keeps_the_replaced_buffer_alive():
    """ops.gemm.workspace grows by replacement; a hipGraph captured with the old buffer keeps
    writing split-K slabs into it on replay (the prefill autotune grows the workspace after
    the decode graphs are captured), so the old buffer must never return to the allocator."""
    from distributed_llm_inferencing_amd.ops import gemm as G
    dev = torch.device("cpu")
    key = (dev.type, dev.index)
    saved, n_ret = G._workspaces.pop(key, None), len(G._retired)
    try:
        small = G.workspace(dev, 1024)
        ptr = small.data_ptr()
        assert G.workspace(dev, 512) is small                 # fits: same buffer
        big = G.workspace(dev, small.numel() + 1)
        assert big is not small and big.numel() > small.numel()
        assert any(t.data_ptr() == ptr for t in G._retired[n_ret:])
    finally:
        del G._retired[n_ret:]
        if saved is not None:
            G._workspaces[key] = saved
        else:
            G._workspaces.pop(key, None)


def test_autotune_final_round_picks_the_lowest_median():
    """ops.gemm._final_round: finalists within the band are re-timed round-robin and the lowest
    median wins, so one lucky first-pass sample cannot pin a plan."""
    from distributed_llm_inferencing_amd.ops import gemm as G
    seq = {"a": iter([1.30, 1.30, 1.30]), "b": iter([1.00, 1.01, 0.99]),
           "c": iter([5.0, 5.0, 5.0])}

    class FakeOps:
        @staticmethod
        def benchmark(run, iters, warmup, graph):
            return next(seq[run()])
    plans = {k: G.GemmPlan("dli", i, 1) for i, k in enumerate("abc")}
    # first pass: "a" got a lucky 0.97 ms, "b" 1.02, "c" far outside the band
    timed = [(0.97, plans["a"], lambda: "a"), (1.02, plans["b"], lambda: "b"),
             (1.5, plans["c"], lambda: "c")]
    best = G._final_round(FakeOps, timed, iters=3, n_copies=1)
    assert best[0] == plans["b"] and abs(best[1] - 1.01) < 1e-9     # median of 4 samples
    assert G._final_round(FakeOps, [], 3, 1) is None
    one = [(2.0, plans["c"], lambda: "c")]
    assert G._final_round(FakeOps, one, 3, 1) == (plans["c"], 2.0)


def test_deferred_norm_plans_and_cpu_gate():
    """Batch-1 reduce-free decode (ops.linear_residual / ops.NormedRows): the "res" epilogue
    is planned over the full-K GEMV tiles only; the prologue tiles are the GEMV tiles; on CPU
    tensors the deferred path is off and a NormedRows input materialises to the reference."""
    from distributed_llm_inferencing_amd import ops
    from distributed_llm_inferencing_amd.ops import gemm as G
    from distributed_llm_inferencing_amd.ops import reference as R
    p1 = G.candidate_plans(1, 4096, 14336, "res")
    assert {p.tile for p in p1} == {30, 32, 56, 57} and {p.splits for p in p1} == {1}
    assert 32 not in {p.tile for p in G.candidate_plans(2, 4096, 4096, "res")}
    assert G._heuristic(1, 4096, 4096, "res") == G.GemmPlan("dli", 56, 1)
    assert G.tile_ok(56, "res") and G.tile_ok(57, "splitk") and not G.tile_ok(56, "silu_mul")
    assert not G.tile_ok(29, "res") and not G.tile_ok(31, "res")
    assert {56, 57} <= {p.tile for p in G.candidate_plans(1, 4096, 4096, "none")}
    assert not {56, 57} & {p.tile for p in G.candidate_plans(8, 4096, 4096, "none")}
    assert set(G.GEMV_PRO_TILES["silu_mul"]) <= set(G.GEMV_TILES)
    torch.manual_seed(0)
    r, nw, w = torch.randn(1, 64).bfloat16(), torch.randn(64).bfloat16(), torch.randn(96, 64).bfloat16()
    assert not ops.deferred_norm_ok(r)
    h = ops.NormedRows(r, nw, 1e-5)
    assert torch.equal(ops.linear(h, w), R.linear(R.rmsnorm(r, nw, 1e-5), w))
    res = torch.randn(1, 96).bfloat16()
    want = res + R.linear(r, w)
    ops.linear_residual(r, w, res)
    assert torch.equal(res, want)
