"""The overlapped decode attention block (models/model.py ``_attn_block_overlapped``): two half
batches on two streams, the second half's split-K scratch in its own workspace slot.

* bitwise equal to running the two halves one after the other on one stream (same kernels,
  same plans), eager and replayed from a captured hipGraph (fork / join in the graph);
* close to the whole-batch path (other GEMM plans: other split-K summation order);
* through the engine: graph decode == eager decode with the overlap on.
"""
import pytest
import torch

from distributed_llm_inferencing_amd import ops
from distributed_llm_inferencing_amd.engine import SamplingParams
from distributed_llm_inferencing_amd.engine.batch import DECODE, DeviceBatch
from distributed_llm_inferencing_amd.engine.llm_engine import LLMEngine
from distributed_llm_inferencing_amd.models import get_config
from distributed_llm_inferencing_amd.models import model as MM
from distributed_llm_inferencing_amd.models.model import TransformerLM
from distributed_llm_inferencing_amd.ops import gemm as G

pytestmark = pytest.mark.gpu
BF = torch.bfloat16


def _decode_setup(gpu, B, seed=0):
    cfg = get_config("llama-tiny128")
    torch.manual_seed(seed)
    model = TransformerLM.random(cfg, device=gpu, seed=seed)
    bs = 16
    lens = torch.randint(1, 60, (B,)).tolist()
    nblk = sum(-(-n // bs) for n in lens) + 4
    shape = (nblk, cfg.num_kv_heads, bs, cfg.head_dim)
    kc = (torch.randn(shape, device=gpu) * 0.5).to(BF)
    vc = (torch.randn(shape, device=gpu) * 0.5).to(BF)
    perm = torch.randperm(nblk).tolist()
    maxb = max(-(-n // bs) for n in lens)
    tables, slots, o = [], [], 0
    for n in lens:
        nb = -(-n // bs)
        blocks = perm[o:o + nb]
        o += nb
        tables.append(blocks + [0] * (maxb - nb))
        slots.append(blocks[(n - 1) // bs] * bs + (n - 1) % bs)
    i32 = dict(device=gpu, dtype=torch.int32)
    batch = DeviceBatch(kind=DECODE, num_seqs=B, num_tokens=B, input_ids=None,
                        positions=torch.tensor([n - 1 for n in lens], **i32),
                        slot_mapping=torch.tensor(slots, **i32),
                        block_tables=torch.tensor(tables, **i32),
                        context_lens=torch.tensor(lens, **i32), max_context=max(lens))
    D = cfg.hidden_size
    h = (torch.randn(B, D, device=gpu) * 0.5).to(BF)
    res = (torch.randn(B, D, device=gpu) * 0.5).to(BF)
    return cfg, model, kc, vc, batch, h, res


def _sequential_halves(model, cfg, lp, batch, h, res, kc, vc, eps):
    B = h.shape[0]
    out = torch.empty_like(h)
    for lo, hi in ((0, B // 2), (B // 2, B)):
        a = ops.linear_rope_attention(
            h[lo:hi], lp["wqkv"], batch.positions[lo:hi], batch.slot_mapping[lo:hi],
            model.cos_sin, kc, vc, batch.block_tables[lo:hi], batch.context_lens[lo:hi],
            batch.max_context, cfg.num_heads, cfg.num_kv_heads, cfg.head_dim, model.scale)
        assert a is not None
        ops.linear_add_rmsnorm(a, lp["wo"], res[lo:hi], lp["mlp_norm"], eps, out=out[lo:hi])
    return out


@pytest.mark.parametrize("splits", [1, 2])
def test_overlapped_attention_block_equals_sequential_halves(gpu, splits):
    B = 16
    cfg, model, kc, vc, batch, h, res = _decode_setup(gpu, B)
    lp, eps = model.layers[0], cfg.norm_eps
    D, Nq = cfg.hidden_size, lp["wqkv"].shape[0]
    for M in (B // 2, B):                 # the same plans for the halves on both sides
        G.set_plan(M, Nq, D, "splitk", G.GemmPlan("dli", 0, splits))
        G.set_plan(M, D, cfg.num_heads * cfg.head_dim, "splitk", G.GemmPlan("dli", 0, 2))
    try:
        kc1, vc1, res1 = kc.clone(), vc.clone(), res.clone()
        ref = _sequential_halves(model, cfg, lp, batch, h, res1, kc1, vc1, eps)
        kc2, vc2, res2 = kc.clone(), vc.clone(), res.clone()
        out = model._attn_block_overlapped(h, lp, batch, kc2, vc2, res2, eps)
        torch.cuda.synchronize()
        assert torch.equal(out, ref) and torch.equal(res2, res1)
        assert torch.equal(kc2, kc1) and torch.equal(vc2, vc1)

        # captured: the fork / join becomes graph edges; replay on fresh copies of the state
        kc3, vc3, res3 = kc.clone(), vc.clone(), res.clone()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):        # warm up (grows both workspace slots)
            model._attn_block_overlapped(h, lp, batch, kc3, vc3, res3, eps)
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        kc3.copy_(kc), vc3.copy_(vc), res3.copy_(res)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            out3 = model._attn_block_overlapped(h, lp, batch, kc3, vc3, res3, eps)
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(out3, ref) and torch.equal(res3, res1)
        assert torch.equal(kc3, kc1) and torch.equal(vc3, vc1)

        # the whole batch at once (its own plan): close, not bitwise
        kc4, vc4, res4 = kc.clone(), vc.clone(), res.clone()
        G.set_plan(B, Nq, D, "splitk", G.GemmPlan("dli", 0, 2 if splits == 1 else 1))
        a = ops.linear_rope_attention(h, lp["wqkv"], batch.positions, batch.slot_mapping,
                                      model.cos_sin, kc4, vc4, batch.block_tables,
                                      batch.context_lens, batch.max_context, cfg.num_heads,
                                      cfg.num_kv_heads, cfg.head_dim, model.scale)
        full = ops.linear_add_rmsnorm(a, lp["wo"], res4, lp["mlp_norm"], eps)
        torch.cuda.synchronize()
        assert (full.float() - ref.float()).abs().max().item() < 0.1
    finally:
        G.clear_plans()


def test_forward_layers_takes_the_overlapped_block(gpu, monkeypatch):
    B = 16
    cfg, model, kc, vc, batch, h, res = _decode_setup(gpu, B, seed=1)
    kv = [(kc.clone(), vc.clone()) for _ in model.layers]
    calls = []
    orig = TransformerLM._attn_block_overlapped

    def spy(self, *a, **k):
        calls.append(a[0].shape[0])
        return orig(self, *a, **k)
    monkeypatch.setattr(TransformerLM, "_attn_block_overlapped", spy)
    monkeypatch.setattr(MM, "OVERLAP", True)
    monkeypatch.setattr(MM, "OVERLAP_MIN", 8)
    out = model.forward_layers(h.clone(), batch, kv)
    torch.cuda.synchronize()
    assert calls == [B] * len(model.layers)
    assert torch.isfinite(out.float()).all()
    calls.clear()
    monkeypatch.setattr(MM, "OVERLAP_MIN", 32)            # below the threshold: not taken
    model.forward_layers(h.clone(), batch, kv)
    assert calls == []


def test_engine_graph_equals_eager_with_overlap(gpu, monkeypatch):
    """16 prompts = the 16-row bucket: eager steps and graph replays split the same rows into
    the same halves under the same (heuristic) plans."""
    monkeypatch.setenv("DLI_GEMM_AUTOTUNE", "0")
    monkeypatch.setattr(MM, "OVERLAP", True)
    monkeypatch.setattr(MM, "OVERLAP_MIN", 16)
    ids = [5, 17, 99, 3, 250, 7, 8, 1000, 42, 11, 600, 3, 3, 9]
    prompts = [ids[i % 9: i % 9 + 5] for i in range(16)]     # equal lengths: B stays 16
    sp = SamplingParams(max_length=32, temperature=0.8, top_k=50, top_p=0.95, seed=5,
                        ignore_eos=True)
    outs = []
    for graphs in (False, True):
        eng = LLMEngine("llama-tiny128", device="cuda", max_batch=16, max_model_len=128,
                        num_blocks=128, use_graphs=graphs, seed=3)
        outs.append([o.output_ids for o in eng.generate(prompts, sp)])
    assert outs[0] == outs[1]
