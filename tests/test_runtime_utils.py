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
