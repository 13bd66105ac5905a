#!/usr/bin/env python3
"""Headline benchmark (BASELINE.json): output tokens/sec (whole node) + p50 request latency,
Llama-3-8B bf16, 1/2/4/8 GPU-workers (layer-sharded pipeline over RCCL for N > 1).

Workload = the reference's request shape (worker/app.py:297-305, views.py:351): synthetic
prompts of --prompt-len random token ids, max_length = 100 tokens INCLUDING the prompt,
do_sample with temperature 0.8 / top_k 50 / top_p 0.95, random-init weights of the real
architecture. EOS is ignored so every request generates exactly max_length - prompt_len
tokens (fixed work per step).

One "step" = one wave of requests served end to end (submit -> last token): --batch
requests per GPU-worker, so per-GPU work is fixed as N grows (weak scaling). N = 1 runs
the single-GPU engine; N > 1 splits the 32 layers into N contiguous stages (one per GPU,
``parallel/pipeline.py``) with N + 1 microbatches of --batch requests in flight.

    python bench.py                               # N=1 defaults
    python bench.py --gpus 8                      # spawns its 8 ranks (launch.py)
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 bench.py --gpus 8

Without torchrun's environment, ``--gpus N > 1`` starts N child ranks itself (one per GPU,
127.0.0.1 rendezvous) before anything touches the GPU, waits for them and exits with the
first failing rank's code. ``DLI_SAME_DEVICE=1`` puts every rank on cuda:0 (a 1-GPU
rehearsal: gloo process group, device-mailbox data plane).

Rank 0 prints one JSON line; multi-rank lines name the resolved data plane (``ipc`` /
``rccl`` / ``torch-rccl`` / ``torch-gloo``), the rank count, every rank's device and the
number of distinct GPUs behind them.
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

METRIC = "output tokens/sec (whole node) + p50 request latency, Llama-3-8B 1/2/4/8 shards"


def _baseline_value():
    """Reference-strategy number measured on MI355X by scripts/bench_reference.py."""
    p = ROOT / "profiles" / "reference_strategy.json"
    if p.exists():
        try:
            return float(json.loads(p.read_text())["value"])
        except Exception:  # noqa: BLE001
            return None
    return None


def _like_for_like_value():
    """HF ``generate`` on 512 prompts per call on MI355X (scripts/bench_reference.py --batch
    512): the batched comparator for the batch-512 row (``vs_baseline`` divides by the
    reference's own strategy, batch 1 serialised)."""
    p = ROOT / "profiles" / "r2_s4" / "hf_generate_b512.json"
    try:
        return float(json.loads(p.read_text())["value"])
    except Exception:  # noqa: BLE001
        return None


def _heartbeat(period_s: float = 45.0):
    """A stderr line every ``period_s`` on rank 0 (stdout keeps the one JSON line): engine
    start-up (weights, autotune, graph capture) and an 8-stage run can stay silent for
    minutes, which a runner's hang detector cannot tell from a stall."""
    import threading
    t0 = time.monotonic()

    def beat():
        while True:
            time.sleep(period_s)
            print(f"[bench] running, {time.monotonic() - t0:.0f} s", file=sys.stderr, flush=True)
    threading.Thread(target=beat, daemon=True, name="bench-heartbeat").start()


def make_prompts(n, prompt_len, vocab, seed):
    # one [n, prompt_len] draw (0.3 ms for 512 x 32) instead of n per-row draws (5.7 ms, a
    # host gap at the head of every timed wave: profiles/r5/s06/wave_summary.txt)
    rng = np.random.default_rng(seed)
    lo, hi = (1000, vocab - 1000) if vocab > 4000 else (3, vocab - 1)
    return rng.integers(lo, hi, size=(n, prompt_len)).tolist()


def run_single(args, barrier=None):
    from distributed_llm_inferencing_amd.engine import SamplingParams
    from distributed_llm_inferencing_amd.engine.llm_engine import LLMEngine

    dev = (torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available()
           else torch.device("cpu"))
    eng = LLMEngine(args.model, device=str(dev), max_batch=args.batch,
                    max_model_len=args.max_model_len, seed=0,
                    max_prefill_tokens=max(args.batch * args.prompt_len, 8192))
    sp = SamplingParams(max_length=args.max_length, temperature=0.8, top_k=50, top_p=0.95,
                        ignore_eos=True)
    eng.warmup()

    def wave(seed):
        prompts = make_prompts(args.batch, args.prompt_len, eng.cfg.vocab_size, seed)
        outs = eng.generate(prompts, sp)
        return sum(len(o.output_ids) for o in outs), [o.latency_s for o in outs]

    for w in range(args.warmup):
        wave(10_000 + w)
    if dev.type == "cuda":
        torch.cuda.synchronize()
    if barrier is not None:
        barrier()
    t0 = time.perf_counter()
    toks, lats = 0, []
    for s in range(args.steps):
        n, l = wave(s)
        toks += n
        lats += l
    if dev.type == "cuda":
        torch.cuda.synchronize()
    if barrier is not None:
        barrier()
    dt = time.perf_counter() - t0
    return {"tokens": toks, "seconds": dt, "latencies": lats, "global_batch": args.batch,
            "parallelism": "single", "engine": eng.stats.snapshot(), "data_plane": "none"}


def run_data_parallel(args, world, rank):
    """Each rank serves its own --batch requests on its own GPU with the single-GPU engine
    (the DP-replica deployment of cli.py serve-cluster); waves are timed between barriers
    and the slowest rank's time is used for the whole-node rate."""
    import torch.distributed as dist
    local = int(os.environ.get("LOCAL_RANK", rank))
    if torch.cuda.is_available():
        torch.cuda.set_device(local)
    from distributed_llm_inferencing_amd.parallel.transport import init_distributed
    init_distributed(device=torch.device("cuda", local) if torch.cuda.is_available() else None)
    res = run_single(args, barrier=dist.barrier)
    cdev = torch.device("cuda", local) if dist.get_backend() == "nccl" else torch.device("cpu")
    t = torch.tensor([res["seconds"], res["tokens"]], dtype=torch.float64, device=cdev)
    mx = t.clone()
    dist.all_reduce(mx, op=dist.ReduceOp.MAX)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    lats = [None] * world
    dist.all_gather_object(lats, res["latencies"])
    from distributed_llm_inferencing_amd.parallel.transport import gather_rank_info
    infos = gather_rank_info(torch.device("cuda", local) if torch.cuda.is_available()
                             else torch.device("cpu"))
    dist.barrier()
    dist.destroy_process_group()
    if rank != 0:
        return None
    return {"tokens": float(t[1].item()), "seconds": float(mx[0].item()),
            "latencies": [x for l in lats for x in l], "global_batch": args.batch * world,
            "parallelism": f"dp{world}", "data_plane": "none", "ranks_info": infos}


def run_pipeline(args, world, rank):
    from distributed_llm_inferencing_amd.models import get_config
    mode = args.mode
    if mode == "auto":
        mode = "ep" if get_config(args.model).is_moe else "pp"
    if mode == "ep":      # Mixtral: DP attention + experts sharded over ranks (all-to-all)
        from distributed_llm_inferencing_amd.parallel.expert import bench_expert_parallel
        return bench_expert_parallel(args, world, rank, make_prompts)
    if mode == "dp":      # N independent replicas (serve-cluster --dp N), no inter-GPU traffic
        return run_data_parallel(args, world, rank)
    if mode == "tp":      # ablation: Megatron-style head/FFN sharding, 2 all-reduces/layer
        from distributed_llm_inferencing_amd.parallel.tensor import bench_tensor_parallel
        return bench_tensor_parallel(args, world, rank, make_prompts)
    from distributed_llm_inferencing_amd.parallel.pipeline import bench_pipeline
    return bench_pipeline(args, world, rank, make_prompts)


def main():
    # every prompt's KV is computed in the timed region: the prompts are random and unique
    # anyway, and prefix caching (on by default for serving) is switched off so that no
    # prefill work could be skipped
    os.environ.setdefault("DLI_PREFIX_CACHE", "0")
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--batch", type=int, default=512, help="requests per microbatch (per GPU-worker) per wave")
    ap.add_argument("--prompt-len", type=int, default=32)
    ap.add_argument("--max-length", type=int, default=100)
    ap.add_argument("--max-model-len", type=int, default=512)
    ap.add_argument("--shard-dir", default=None,
                    help="N>1 pp: load each stage from <dir>/shard_<rank>/ (shard-model output)")
    ap.add_argument("--pp-prefill-chunks", type=int, default=2,
                    help="N>1 pp: admit each microbatch's prompts over this many prefill "
                         "steps (smaller ring-fill bubble at the start of a wave)")
    ap.add_argument("--mode", default="auto", choices=["auto", "pp", "ep", "tp", "dp"],
                    help="N>1: pp = layer-sharded pipeline (dense, default), ep = expert "
                         "parallel (MoE), tp = tensor-parallel ablation, dp = independent "
                         "replicas")
    a = ap.parse_args()

    from distributed_llm_inferencing_amd import launch
    if a.gpus > 1 and not launch.under_launcher():
        # the plain form `python bench.py --gpus N`: start the N ranks here, before any GPU
        # call in this process (counting devices does not initialise HIP)
        n_dev = launch.visible_gpus()
        if 0 < n_dev < a.gpus and os.environ.get("DLI_SAME_DEVICE", "0") != "1":
            sys.exit(f"bench.py: --gpus {a.gpus} but only {n_dev} GPU(s) visible "
                     "(DLI_SAME_DEVICE=1 rehearses every rank on cuda:0)")
        sys.exit(launch.spawn_self(a.gpus))

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if rank == 0:
        _heartbeat()
    if world > 1 or a.gpus > 1:
        res = run_pipeline(a, world, rank)
    else:
        res = run_single(a)
    if rank != 0 or res is None:
        return
    tok_s = res["tokens"] / res["seconds"]
    p50 = statistics.median(res["latencies"]) if res["latencies"] else None
    base = _baseline_value()
    line = {
        "metric": METRIC,
        "value": round(tok_s, 2),
        "unit": "tokens/s",
        "n_gpus": max(a.gpus, world),
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(1000 * res["seconds"] / max(1, a.steps), 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": round(tok_s / base, 3) if base else None,
        "baseline_note": "vs_baseline = value / the reference's strategy measured on MI355X "
                         "(HF generate, batch 1, serialised: profiles/reference_strategy.json)",
        "dtype": "bf16",
        "data": "synthetic prompts, random-init weights",
        "p50_latency_s": round(p50, 4) if p50 is not None else None,
        "config": {"model": a.model, "global_batch": res["global_batch"],
                   "seq_len": a.max_length, "prompt_len": a.prompt_len,
                   "parallelism": res["parallelism"],
                   "sampling": "T=0.8 top_k=50 top_p=0.95"},
        "data_plane": res.get("data_plane", "none"),
        "ranks": world,
        "launcher": os.environ.get("DLI_LAUNCHER", "torchrun" if world > 1 else "none"),
    }
    eng = res.get("engine") or {}
    keep = ("head_host_ms_per_tick", "head_host_ms_per_decode_tick", "head_phase_ms_per_tick",
            "lockstep_ms_per_step", "control_plane", "decode_steps", "prefill_steps", "steps")
    if any(k in eng for k in keep[:4]):
        # multi-rank pipeline: the head's host cost per tick (it schedules every microbatch)
        line["engine"] = {k: eng[k] for k in keep if k in eng}
    infos = res.get("ranks_info")
    if infos:
        from distributed_llm_inferencing_amd.parallel.transport import distinct_gpus
        line["rank_devices"] = [{k: i[k] for k in ("rank", "device", "pci", "host")
                                 if k in i} for i in infos]
        line["distinct_gpus"] = distinct_gpus(infos)
    lfl = _like_for_like_value()
    if lfl and a.model == "llama3-8b":
        # like-for-like batch: HF generate over 512 prompts per call on the same GPU
        line["vs_hf_batched_generate"] = round(tok_s / lfl, 3)
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
