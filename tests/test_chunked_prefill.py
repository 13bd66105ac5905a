"""Chunked prefill (SURVEY.md §5.7 long context; VERDICT r1 'What's missing' 7): prompts longer
than ``max_prefill_tokens`` are prefilled over several steps, each chunk attending over the
paged cache (earlier chunks + itself). Outputs must be token-identical to whole-prompt
prefill, also when chunks interleave with decode steps of running sequences and after
preemption recomputes."""
import numpy as np
import pytest
import torch

from distributed_llm_inferencing_amd.engine import SamplingParams
from distributed_llm_inferencing_amd.engine.llm_engine import LLMEngine
from distributed_llm_inferencing_amd.ops import reference as R

PROMPTS = [list(range(3, 3 + 45)), [7, 8, 9], list(range(100, 100 + 70)), [5] * 17,
           list(range(200, 233))]


def _engine(chunk, **kw):
    kw.setdefault("num_blocks", 256)
    return LLMEngine("llama-tiny", device="cpu", dtype=torch.float32, max_batch=8,
                     max_model_len=256, max_prefill_tokens=chunk, **kw)


def test_paged_reference_matches_contiguous():
    torch.manual_seed(0)
    hq, hkv, hd, bs = 4, 2, 16, 4
    lens = [5, 11, 1]
    T = sum(lens)
    q = torch.randn(T, hq, hd)
    k = torch.randn(T, hkv, hd)
    v = torch.randn(T, hkv, hd)
    cu = torch.tensor([0, 5, 16, 17], dtype=torch.int32)
    want = R.prefill_attention(q, k, v, cu, 0.25)
    # scatter K/V into a shuffled paged cache, then attend chunk = whole prompt (ctx = len)
    nblk = 16
    kc = torch.zeros(nblk, hkv, bs, hd)
    vc = torch.zeros(nblk, hkv, bs, hd)
    perm = torch.randperm(nblk).tolist()
    tables = torch.zeros(3, 4, dtype=torch.int32)
    nxt = 0
    for i, L in enumerate(lens):
        for b in range(-(-L // bs)):
            tables[i, b] = perm[nxt]
            nxt += 1
        for t in range(L):
            blk = int(tables[i, t // bs])
            kc[blk, :, t % bs] = k[int(cu[i]) + t]
            vc[blk, :, t % bs] = v[int(cu[i]) + t]
    got = R.prefill_attention_paged(q, kc, vc, cu, torch.tensor(lens), tables, 0.25)
    torch.testing.assert_close(got, want, rtol=1e-5, atol=1e-5)
    # the last 4 queries of sequence 1 as a chunk over its 11 cached keys
    qc = q[int(cu[1]) + 7:int(cu[1]) + 11]
    got_c = R.prefill_attention_paged(qc, kc, vc, torch.tensor([0, 4], dtype=torch.int32),
                                      torch.tensor([11]), tables[1:2], 0.25)
    torch.testing.assert_close(got_c, want[int(cu[1]) + 7:int(cu[1]) + 11], rtol=1e-5,
                               atol=1e-5)


@pytest.mark.parametrize("chunk", [16, 40])
def test_chunked_prefill_token_identical(chunk):
    ref = _engine(4096)
    eng = _engine(chunk)
    for sp in (SamplingParams(max_length=90, do_sample=False, ignore_eos=True),
               SamplingParams(max_length=90, seed=5, ignore_eos=True)):
        want = [o.all_ids for o in ref.generate(PROMPTS, sp)]
        got = [o.all_ids for o in eng.generate(PROMPTS, sp)]
        assert got == want
    assert eng.stats.prefill_steps > ref.stats.prefill_steps
    assert not any(eng.scheduler.prefilling)


@pytest.mark.parametrize("mixed", [False, True])
def test_chunks_interleave_with_decode(mixed):
    """A long prompt submitted while short requests decode: the running sequences keep
    producing tokens and every output is unchanged. Without mixed steps the chunks alternate
    with decode steps; with them every chunk step also carries the decode rows."""
    sp = SamplingParams(max_length=60, do_sample=False, ignore_eos=True)
    long_p = list(range(10, 10 + 150))
    ref = _engine(4096)
    want_short = [o.all_ids for o in ref.generate(PROMPTS[1:2] + PROMPTS[3:4], sp)]
    want_long = ref.generate([long_p], SamplingParams(max_length=170, do_sample=False,
                                                       ignore_eos=True))[0].all_ids
    eng = _engine(16, mixed_steps=mixed)
    rids = [eng.add_request(p, sp) for p in (PROMPTS[1], PROMPTS[3])]
    for _ in range(3):
        eng.step()
    rid_long = eng.add_request(long_p, SamplingParams(max_length=170, do_sample=False,
                                                      ignore_eos=True))
    kinds = []
    outs = {}
    while eng.has_work():
        meta = eng.plan_step()
        if meta is not None:
            kinds.append((meta.kind, bool(meta.sample_mask is not None), meta.num_decode))
        for o in eng.finish_step(meta):
            outs[o.request_id] = o
    assert [outs[r].all_ids for r in rids] == want_short
    assert outs[rid_long].all_ids == want_long
    chunk_steps = [i for i, (k, partial, _) in enumerate(kinds) if k == 1 and partial]
    assert len(chunk_steps) >= 8                       # 150 tokens in 16-token chunks
    if mixed:
        # back-to-back chunk steps, each with both short requests' decode rows
        assert np.diff(chunk_steps[:3]).tolist() == [1, 1], kinds[:20]
        assert all(kinds[i][2] == 2 for i in chunk_steps[:3]), kinds[:20]
        assert eng.stats.mixed_steps >= 3
    else:
        # while the short requests still decode, no two chunk steps are adjacent
        gaps = np.diff(chunk_steps[:3])
        assert (gaps >= 2).all(), kinds[:20]
        assert eng.stats.mixed_steps == 0


def test_chunked_prefill_with_preemption():
    sp = SamplingParams(max_length=120, do_sample=False, ignore_eos=True)
    prompts = [list(range(20 + i, 20 + i + 40)) for i in range(6)]
    ref = _engine(4096)
    want = [o.all_ids for o in ref.generate(prompts, sp)]
    eng = _engine(24, num_blocks=40)                   # 160 tokens of KV: forces preemption
    n_pre = [0]
    orig = eng.scheduler._preempt

    def counted(mb):
        n_pre[0] += 1
        return orig(mb)
    eng.scheduler._preempt = counted
    got = [o.all_ids for o in eng.generate(prompts, sp)]
    assert got == want
    assert n_pre[0] > 0
