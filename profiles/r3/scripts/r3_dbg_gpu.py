import sys, torch, numpy as np
sys.path.insert(0, '.')
from distributed_llm_inferencing_amd import ops
from distributed_llm_inferencing_amd.ops import gemm as G, reference as R
dev = torch.device('cuda')
torch.manual_seed(0)
for (M, N, K) in [(1, 1024, 256), (1, 4096, 4096), (2, 512, 1024)]:
    x = torch.randn(M, K, device=dev).to(torch.bfloat16)
    w = (torch.randn(N, K, device=dev) * 0.05).to(torch.bfloat16)
    ref = R.linear(x, w, out_dtype=torch.float32)
    for tile in (30, 31):
        out = ops._gemm_native(x, w, "f32", plan=G.GemmPlan("dli", tile, 1))
        torch.cuda.synchronize()
        print(M, N, K, tile, "maxerr", (out - ref).abs().max().item(), "refmax", ref.abs().max().item(), flush=True)
# to_device check
from distributed_llm_inferencing_amd.engine.batch import to_device, StepMeta, PREFILL
T = 7
m = StepMeta(kind=PREFILL, seq_ids=[0], input_ids=np.arange(5, 5 + T, dtype=np.int32), positions=np.arange(T, dtype=np.int32),
             slot_mapping=-np.ones(T, np.int32), seq_lens=np.array([T], np.int32), context_lens=np.array([T], np.int32),
             block_tables=np.zeros((1, 0), np.int32), temperature=np.zeros(1, np.float32), top_k=np.ones(1, np.int32),
             top_p=np.ones(1, np.float32), seeds=np.array([123456789012], np.int64))
db = to_device(m, dev)
cdb = to_device(m, 'cpu')
for f in ("input_ids", "positions", "slot_mapping", "temperature", "top_k", "top_p", "seeds", "cu_seqlens", "last_token_idx"):
    a, b = getattr(db, f), getattr(cdb, f)
    print(f, a.cpu().tolist(), b.tolist(), a.dtype, flush=True)
