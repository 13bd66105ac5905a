"""Mixed prefill+decode steps: when prompts arrive while a microbatch is decoding, the
prefill step also carries every running sequence's decode row (decode rows first, attended by
the decode kernel; prompt rows by the paged prefill kernel). Outputs must be token-identical
to the engine without mixed steps, with lookahead on and off, with stop tokens that end a
sequence inside an in-flight step, and with chunked prompts."""
import pytest
import torch

from distributed_llm_inferencing_amd.engine import SamplingParams
from distributed_llm_inferencing_amd.engine.llm_engine import LLMEngine

WAVES = [
    [[5, 6, 7, 8], [9, 10, 11], list(range(30, 52))],
    [[100, 200], [7] * 9],
    [list(range(60, 100)), [3, 4]],
]


def _engine(mixed, lookahead, chunk=4096, model="llama-tiny"):
    return LLMEngine(model, device="cpu", dtype=torch.float32, max_batch=8,
                     max_model_len=128, num_blocks=128, max_prefill_tokens=chunk,
                     mixed_steps=mixed, lookahead=lookahead)


def _run(eng, params):
    """Submit WAVES[0], step twice, submit WAVES[1], step once, submit WAVES[2], drain."""
    outs, rids, k = {}, [], 0
    for w, wave in enumerate(WAVES):
        for p in wave:
            rids.append(eng.add_request(p, params[k]))
            k += 1
        for _ in range((2, 1, 0)[w]):
            for o in eng.step():
                outs[o.request_id] = o
    while eng.has_work():
        for o in eng.step():
            outs[o.request_id] = o
    return [(outs[r].all_ids, outs[r].finish_reason) for r in rids]


@pytest.mark.parametrize("lookahead", [True, False])
@pytest.mark.parametrize("chunk", [4096, 16])
def test_mixed_steps_token_identical(lookahead, chunk):
    n = sum(len(w) for w in WAVES)
    greedy = [SamplingParams(max_length=40 + 3 * i, do_sample=False, ignore_eos=True)
              for i in range(n)]
    sampled = [SamplingParams(max_length=36, seed=100 + i, ignore_eos=True) for i in range(n)]
    for params in (greedy, sampled):
        want = _run(_engine(False, lookahead, chunk), params)
        eng = _engine(True, lookahead, chunk)
        got = _run(eng, params)
        assert got == want
        assert eng.stats.mixed_steps > 0
        assert eng.stats.tokens_out == sum(len(a) - len(p) for (a, _), p in
                                           zip(got, [p for w in WAVES for p in w]))


def test_mixed_steps_with_stop_tokens():
    """A sequence that stops on a stop token while its next row is already scheduled (the
    in-flight step under lookahead) loses that row's token in both engines alike."""
    n = sum(len(w) for w in WAVES)
    base = [SamplingParams(max_length=44, do_sample=False, ignore_eos=True) for _ in range(n)]
    free = _run(_engine(False, True), base)
    params = []
    for (ids, _), p in zip(free, [p for w in WAVES for p in w]):
        gen = ids[len(p):]
        stop = [gen[len(gen) // 3]] if len(gen) > 3 else []
        params.append(SamplingParams(max_length=44, do_sample=False, ignore_eos=True,
                                     stop_token_ids=stop))
    want = _run(_engine(False, True), params)
    assert any(r == "stop" for _, r in want)
    eng = _engine(True, True)
    assert _run(eng, params) == want
    assert eng.stats.mixed_steps > 0


@pytest.mark.parametrize("model", ["gpt2-tiny", "mixtral-tiny"])
def test_mixed_steps_other_families(model):
    """GPT-2 (learned positions, LayerNorm, no RoPE) and Mixtral (routed experts over the
    mixed rows) through mixed steps."""
    n = sum(len(w) for w in WAVES)
    params = [SamplingParams(max_length=36, seed=300 + i, ignore_eos=True) for i in range(n)]
    want = _run(_engine(False, True, model=model), params)
    eng = _engine(True, True, model=model)
    assert _run(eng, params) == want
    assert eng.stats.mixed_steps > 0


def test_mixed_step_metadata_survives_the_wire():
    """A mixed step crosses pipeline stages as packed metadata: the decode-row count rides
    in header word 9 (both the generic and the native-decode packing paths)."""
    import numpy as np

    from distributed_llm_inferencing_amd.engine.batch import PREFILL, StepMeta
    S, T = 3, 7
    m = StepMeta(kind=PREFILL, seq_ids=[4, 9, 11], input_ids=np.arange(T, dtype=np.int32),
                 positions=np.arange(T, dtype=np.int32), slot_mapping=np.arange(T, dtype=np.int32),
                 seq_lens=np.array([1, 1, 5], np.int32), context_lens=np.array([9, 4, 5], np.int32),
                 block_tables=np.array([[1, 2], [3, 0], [4, 0]], np.int32),
                 temperature=np.full(S, 0.8, np.float32), top_k=np.full(S, 50, np.int32),
                 top_p=np.full(S, 0.95, np.float32), seeds=np.arange(S, dtype=np.int64),
                 microbatch=2, step_id=17, num_decode=2)
    h, p = m.pack()
    assert int(h[9]) == 2
    u = StepMeta.unpack(h, p)
    assert u.num_decode == 2 and u.kind == PREFILL and u.seq_ids == [4, 9, 11]
    assert np.array_equal(u.block_tables, m.block_tables)
    m.num_decode = 0
    assert StepMeta.unpack(*m.pack()).num_decode == 0


@pytest.mark.parametrize("lookahead", [True, False])
def test_mixed_steps_under_preemption(lookahead):
    """KV pressure with mixed steps + lookahead + a non-empty waiting queue: a sequence the
    decode half of a mixed step preempts must not be re-admitted by that same step's prefill
    half (its in-flight token would then be applied twice). Outputs must equal an
    unconstrained run's."""
    n = sum(len(w) for w in WAVES)
    params = [SamplingParams(max_length=60, do_sample=False, ignore_eos=True) for _ in range(n)]
    want = _run(_engine(False, False), params)
    eng = LLMEngine("llama-tiny", device="cpu", dtype=torch.float32, max_batch=8,
                    max_model_len=128, num_blocks=14, block_size=16, max_prefill_tokens=4096,
                    mixed_steps=True, lookahead=lookahead)
    got = _run(eng, params)
    assert eng.scheduler.num_preempted > 0 and eng.stats.mixed_steps > 0
    assert got == want
