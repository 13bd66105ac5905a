"""Multi-process pipeline (PP) and expert-parallel (EP) exchanges with GPU tensors: 2 ranks
share cuda:0 over gloo (RCCL refuses two ranks on one GPU). The data plane, the shared-memory
control ring, the hipGraph stage runners and the EP buckets all run on device memory here,
so the only thing the 8-GPU driver run adds is the RCCL transport itself.
Each rank's output must equal the single-process engine's, token for token."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from distributed_llm_inferencing_amd.engine import SamplingParams
from distributed_llm_inferencing_amd.engine.llm_engine import LLMEngine

pytestmark = pytest.mark.gpu
PROMPTS = [[5, 6, 7, 8], [9, 10, 11], [1, 2, 3, 4, 5, 6, 7], [100, 200], [7] * 9, [3, 4], [8] * 3]
GREEDY = SamplingParams(max_length=24, do_sample=False, ignore_eos=True)
SAMPLED = SamplingParams(max_length=24, seed=11, ignore_eos=True)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _env(rank, world, port, **extra):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank), DLI_DIST_BACKEND="gloo",
                      DLI_SAME_DEVICE="1", DLI_GEMM_AUTOTUNE="0", **extra)


def _pp_worker(rank, world, port, q, vp, comm="torch"):
    # comm "auto": no data-plane override at all (the default must resolve to the mailboxes)
    _env(rank, world, port, DLI_PP_VOCAB_PARALLEL=vp,
         **({} if comm == "auto" else {"DLI_PP_COMM": comm}))
    if comm == "auto":
        os.environ.pop("DLI_PP_COMM", None)
    import torch.distributed as dist
    from distributed_llm_inferencing_amd.parallel.pipeline import DistributedPipelineEngine
    eng = DistributedPipelineEngine("llama-tiny", "cuda", max_batch=8, max_model_len=64,
                                    num_blocks=256)
    x0 = 0
    if comm == "auto":
        assert eng.channel.comm == "ipc" and eng.channel.ipc.mem_kind == "uncached"
        eng.warmup()                  # captures the receive / send into the decode graphs
        x0 = eng.channel.exchanges    # captured calls counted once, at capture
    if rank == 0:
        res = [[o.all_ids for o in eng.generate(PROMPTS, sp)] for sp in (GREEDY, SAMPLED)]
        res.append(eng.vocab_parallel)
        res.append(eng.channel.ipc.stats() if eng.channel.ipc is not None else None)
        eng.shutdown()
        q.put(res)
    else:
        eng.serve()
    if rank != 0 and comm == "auto":
        from distributed_llm_inferencing_amd.engine.batch import DECODE, PREFILL
        run = eng.stage.runner
        q.put(("stage", rank, run.piped is not None, run.replays, run.uploads,
               eng.stage.tick_counts.get(DECODE, 0), eng.stage.tick_counts.get(PREFILL, 0),
               eng.channel.exchanges - x0))
    dist.barrier()
    eng.channel.close()
    dist.destroy_process_group()


def _run(target, world, *args):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, q) + args) for r in range(world)]
    for p in procs:
        p.start()
    try:
        n = world if (target in (_ep_worker, _ep_ipc_worker) or "auto" in args) else 1
        res = [q.get(timeout=240) for _ in range(n)]
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    return res


@pytest.mark.timeout(300)
@pytest.mark.parametrize("vp", ["0", "1"])
def test_pipeline_two_ranks_on_gpu_match_single_stage(gpu, vp):
    """2-stage pipeline over gloo on GPU tensors (tail LM head, and the vocab-parallel head
    with the HIP per-slice top-k) == the single-stage engine."""
    (res,) = _run(_pp_worker, 2, vp)
    os.environ["DLI_GEMM_AUTOTUNE"] = "0"
    try:
        eng = LLMEngine("llama-tiny", device="cuda", max_batch=8, max_model_len=64,
                        num_blocks=64)
        assert res[0] == [o.all_ids for o in eng.generate(PROMPTS, GREEDY)]
        assert res[1] == [o.all_ids for o in eng.generate(PROMPTS, SAMPLED)]
    finally:
        del os.environ["DLI_GEMM_AUTOTUNE"]
    assert res[2] == (vp == "1")


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world,vp", [(2, "0"), (2, "1"), (4, "0"), (4, "1")])
def test_pipeline_over_ipc_mailboxes_on_gpu(gpu, world, vp):
    """The DEFAULT data plane (no DLI_PP_COMM) with N ranks on ONE GPU resolves to the
    device mailboxes: every activation / token / candidate message goes through
    hipIpc-mapped uncached mailboxes (stream-ordered put / get kernels with sequence-checked
    headers, bounded wait / signal kernels, csrc/runtime/ipc.cpp), token-identical to the
    single-stage engine."""
    out = _run(_pp_worker, world, vp, "auto")
    (res,) = [x for x in out if x[0] != "stage"]
    stages = [x for x in out if x[0] == "stage"]
    assert len(stages) == world - 1
    for _, rank, piped, replays, uploads, dec, pre, exch in stages:
        assert piped                                  # receive/send captured in the graphs
        # one metadata H2D + one graph launch per decode tick, nothing else on the data
        # plane: the only eager exchanges are the prefill ticks' receive + send (and the
        # vocab-parallel side messages on the tail / candidates)
        assert replays == dec and uploads == dec and dec > 0, (rank, replays, uploads, dec)
        if vp == "0":
            assert exch <= 2 * pre + 1, (rank, exch, pre)
    os.environ["DLI_GEMM_AUTOTUNE"] = "0"
    try:
        eng = LLMEngine("llama-tiny", device="cuda", max_batch=8, max_model_len=64,
                        num_blocks=64)
        assert res[0] == [o.all_ids for o in eng.generate(PROMPTS, GREEDY)]
        assert res[1] == [o.all_ids for o in eng.generate(PROMPTS, SAMPLED)]
    finally:
        del os.environ["DLI_GEMM_AUTOTUNE"]
    assert res[2] == (vp == "1")
    assert res[3]["sends"] > 0 and res[3]["recvs"] > 0 and res[3]["bytes_out"] > 0


def _ep_worker(rank, world, port, q):
    _env(rank, world, port, DLI_EP_COMM="torch")
    import torch.distributed as dist
    from distributed_llm_inferencing_amd.parallel.expert import ExpertParallelEngine
    eng = ExpertParallelEngine("mixtral-tiny", "cuda", max_batch=8, max_model_len=64,
                               num_blocks=64)
    mine = PROMPTS[rank::world]
    out = [o.all_ids for o in eng.generate(mine, GREEDY)]
    q.put((rank, mine, out, eng.moe.host_reads, eng.lockstep_syncs, eng.steps,
           eng.engine.lookahead))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_expert_parallel_two_ranks_on_gpu_match_dense(gpu):
    """DP attention + experts split over 2 ranks (ep_pack buckets, grouped GEMMs, moe_combine
    on the GPU, exchanged over gloo) == one process holding all experts; no routing value
    read on the host on any step, one lockstep sync per step."""
    res = _run(_ep_worker, 2)
    os.environ["DLI_GEMM_AUTOTUNE"] = "0"
    try:
        eng = LLMEngine("mixtral-tiny", device="cuda", max_batch=8, max_model_len=64,
                        num_blocks=64)
        for rank, mine, out, reads, syncs, steps, la in res:
            assert out == [o.all_ids for o in eng.generate(mine, GREEDY)], rank
            assert reads == 0 and syncs == steps + 1 and la
    finally:
        del os.environ["DLI_GEMM_AUTOTUNE"]


def _ep_ipc_worker(rank, world, port, q):
    _env(rank, world, port)
    os.environ.pop("DLI_EP_COMM", None)          # the default must resolve to the mailboxes
    import torch.distributed as dist
    from distributed_llm_inferencing_amd.parallel.expert import ExpertParallelEngine
    eng = ExpertParallelEngine("mixtral-tiny", "cuda", max_batch=8, max_model_len=64,
                               num_blocks=64)
    assert eng.comm == "ipc" and eng.moe.ep.mem_kind == "uncached"
    eng.warmup()                      # every decode bucket captured, exchanges included
    mine = PROMPTS[rank::world]
    out = [o.all_ids for o in eng.generate(mine, GREEDY)]
    q.put((rank, mine, out, eng.graph_steps, eng.lockstep_syncs, eng.steps,
           eng.engine.runner.uploads, eng.engine.lookahead))
    dist.barrier()
    eng.moe.close()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("world", [2, 4])
def test_expert_parallel_over_ipc_graphs_on_gpu(gpu, world):
    """Experts over N ranks on one GPU through the IPC mailboxes: counts stay on the device,
    the decode forward (attention + every MoE dispatch / return) is one graph replay, one
    lockstep sync per step; tokens identical to one process holding every expert."""
    res = _run(_ep_ipc_worker, world)
    os.environ["DLI_GEMM_AUTOTUNE"] = "0"
    try:
        eng = LLMEngine("mixtral-tiny", device="cuda", max_batch=8, max_model_len=64,
                        num_blocks=64)
        for rank, mine, out, graph_steps, syncs, steps, uploads, la in res:
            assert out == [o.all_ids for o in eng.generate(mine, GREEDY)], rank
            assert syncs == steps + 1 and la
            assert graph_steps > 0 and uploads == graph_steps   # one H2D + one replay
    finally:
        del os.environ["DLI_GEMM_AUTOTUNE"]


def _register_16l():
    from dataclasses import replace
    from distributed_llm_inferencing_amd.models.configs import get_config, register
    register(replace(get_config("llama3-8b"), name="llama3-8b-16l", num_layers=16))


def _pp8_worker(rank, world, port, q):
    _env(rank, world, port)
    os.environ.pop("DLI_PP_COMM", None)          # the default plane: the IPC mailboxes
    os.environ.pop("DLI_PP_VOCAB_PARALLEL", None)  # the default head at N >= 4: vocab-parallel
    _register_16l()
    import torch.distributed as dist
    from distributed_llm_inferencing_amd.parallel.pipeline import DistributedPipelineEngine
    eng = DistributedPipelineEngine("llama3-8b-16l", "cuda", max_batch=8, max_model_len=64,
                                    num_blocks=64)
    assert eng.channel.comm == "ipc" and eng.vocab_parallel
    assert eng.stage.plan.end_layer - eng.stage.plan.start_layer == 2
    eng.warmup()
    if rank == 0:
        q.put([o.all_ids for o in eng.generate(PROMPTS, GREEDY)])
        eng.shutdown()
    else:
        eng.serve()
    dist.barrier()
    eng.channel.close()
    dist.destroy_process_group()


@pytest.mark.timeout(420)
def test_pipeline_pp8_real_shape_stages_match_single_engine(gpu):
    """The driver's 8-rank pipeline form at the real Llama-3-8B layer shapes (d 4096, 32 q /
    8 kv heads, FFN 14336, vocab 128256), 2 layers per stage, all 8 ranks on cuda:0: default
    data plane (IPC mailboxes), vocab-parallel head, M = 11 microbatches, decode graphs with
    the captured receive / send — greedy tokens identical to one engine holding all 16
    layers."""
    (res,) = _run(_pp8_worker, 8)
    _register_16l()
    os.environ["DLI_GEMM_AUTOTUNE"] = "0"
    try:
        eng = LLMEngine("llama3-8b-16l", device="cuda", max_batch=8, max_model_len=64,
                        num_blocks=64)
        assert res == [o.all_ids for o in eng.generate(PROMPTS, GREEDY)]
    finally:
        del os.environ["DLI_GEMM_AUTOTUNE"]
