"""Lookahead scheduling (engine/llm_engine.py, engine/scheduler.py): the single-stage engine
schedules and launches step k+1 before the tokens of step k reach the host; the next step's
input ids come from the in-flight step's device output. Outputs must be token-identical to the
synchronous engine — greedy and sampled, with stop tokens ending sequences one step after they
were scheduled again, and with preemption under KV pressure."""
import numpy as np
import pytest
import torch

from distributed_llm_inferencing_amd.engine import SamplingParams
from distributed_llm_inferencing_amd.engine.llm_engine import LLMEngine
from distributed_llm_inferencing_amd.engine.scheduler import Scheduler
from distributed_llm_inferencing_amd.runtime import BlockManager

PROMPTS = [[i + 3] * (4 + i % 5) for i in range(6)]


def _run(lookahead, sp, num_blocks=64, prompts=PROMPTS):
    eng = LLMEngine("llama-tiny", device="cpu", dtype=torch.float32, max_batch=8,
                    max_model_len=64, num_blocks=num_blocks, seed=5, lookahead=lookahead)
    outs = eng.generate(prompts, sp)
    assert eng.bm.num_free == num_blocks          # every block returned
    assert not eng.has_work()
    return [(o.all_ids, o.finish_reason) for o in outs]


@pytest.mark.parametrize("sp", [
    SamplingParams(max_length=40, do_sample=False, ignore_eos=True),
    SamplingParams(max_length=40, seed=7, ignore_eos=True),
    SamplingParams(max_new_tokens=9, seed=3),
])
def test_lookahead_matches_synchronous(sp):
    assert _run(True, sp) == _run(False, sp)


def test_lookahead_with_stop_tokens_matches_synchronous():
    """Stops the lookahead cannot predict: tokens the synchronous run samples become stop
    tokens, so sequences end while their next step is already scheduled."""
    sp = SamplingParams(max_length=40, seed=11, ignore_eos=True)
    ref = _run(False, sp)
    stops = sorted({ids[len(p) + 4] for (ids, _), p in zip(ref, PROMPTS)})
    sp2 = SamplingParams(max_length=40, seed=11, ignore_eos=True, stop_token_ids=stops)
    got = _run(True, sp2)
    assert got == _run(False, sp2)
    assert any(r == "stop" for _, r in got)


def test_lookahead_under_kv_pressure_matches_synchronous():
    sp = SamplingParams(max_length=48, do_sample=False, ignore_eos=True)
    prompts = [[i + 3] * 8 for i in range(4)]
    assert _run(True, sp, num_blocks=8, prompts=prompts) == \
        _run(False, sp, num_blocks=8, prompts=prompts)


def test_scheduler_schedules_one_step_ahead():
    """The decode scheduled against an in-flight step advances its sequences by one token,
    leaves out those the in-flight token completes and feeds ids from its output rows."""
    bm = BlockManager(64, 16)
    s = Scheduler(bm, max_seqs_per_mb=8, max_model_len=64)
    s.add_request("a", [1, 2, 3], SamplingParams(max_new_tokens=1))
    s.add_request("b", [4, 5], SamplingParams(max_new_tokens=5))
    pre = s.schedule(0)
    assert pre.kind == 1 and pre.num_seqs == 2
    nxt = s.schedule(0, inflight=pre)
    # "a" finishes with the prefill's token; "b" decodes at position 2 with its fed id
    assert nxt.kind == 2 and nxt.seq_ids == [pre.seq_ids[1]]
    assert nxt.positions.tolist() == [2] and nxt.context_lens.tolist() == [3]
    assert nxt.feed_src.tolist() == [1]
    s.update(pre, np.array([7, 8], np.int32))
    assert [q.request_id for q in s.pop_finished()] == ["a"]
    s.update(nxt, np.array([9], np.int32))
    assert s.seqs[pre.seq_ids[1]].output_ids == [8, 9]


def test_admission_window_batches_trickling_arrivals():
    """While decoding, a lone arrival waits (up to the window) for more arrivals instead of
    triggering a one-request prefill; after the window it is admitted; with nothing running
    it is admitted at once."""
    import time
    bm = BlockManager(256, 16)
    s = Scheduler(bm, max_seqs_per_mb=16, max_model_len=128, admit_window_s=0.05,
                  admit_min_frac=0.25)                       # want 4 arrivals
    s.add_request("a", [1, 2, 3], SamplingParams(max_new_tokens=50))
    m = s.schedule(0)
    assert m.kind == 1                                        # idle engine: admitted at once
    s.update(m, np.array([5], np.int32))
    s.add_request("b", [4, 5], SamplingParams(max_new_tokens=50))
    assert s.schedule(0).kind == 2                            # decode; "b" waits
    for i in range(3):
        s.add_request(f"c{i}", [6, 7], SamplingParams(max_new_tokens=50))
    m = s.schedule(0)
    assert m.kind == 1 and m.num_seqs == 4                    # batch of 4 arrivals
    s.update(m, np.arange(4, dtype=np.int32) + 3)
    s.add_request("d", [8], SamplingParams(max_new_tokens=5))
    assert s.schedule(0).kind == 2
    time.sleep(0.06)
    m = s.schedule(0)
    assert m.kind == 1 and m.num_seqs == 1                    # window expired


def test_refill_pacing_when_nearly_full():
    """More requests in flight than slots: a nearly full microbatch (fewer free slots than
    admit_min) refills at most once per refill interval instead of running a prefill step
    after every decode step that frees a slot or two; with admit_min free slots it refills
    at once."""
    import time
    bm = BlockManager(512, 16)
    s = Scheduler(bm, max_seqs_per_mb=16, max_model_len=128, admit_window_s=0.01,
                  admit_min_frac=0.25, refill_interval_s=0.05)     # admit_min = 4
    for i in range(14):
        s.add_request(f"r{i}", [1, 2], SamplingParams(max_new_tokens=2 if i < 1 else 60))
    m = s.schedule(0)
    assert m.kind == 1 and m.num_seqs == 14
    s.update(m, np.full(14, 3, np.int32))
    for i in range(6):
        s.add_request(f"q{i}", [4, 5], SamplingParams(max_new_tokens=60))
    time.sleep(0.02)                                   # queued longer than the window
    m = s.schedule(0)
    assert m.kind == 2                                 # 2 free slots < 4: paced
    s.update(m, np.full(m.num_seqs, 3, np.int32))      # r0 finishes: 3 free
    assert s.schedule(0).kind == 2
    time.sleep(0.05)
    m = s.schedule(0)
    assert m.kind == 1 and m.num_seqs == 3             # interval passed: refill the 3 slots
