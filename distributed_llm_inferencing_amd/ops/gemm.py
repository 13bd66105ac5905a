"""GEMM planning: tile shape / split-K choice for the MFMA kernel, plus optional autotune.

The projection GEMMs of a decode step are skinny (M = batch) and of a prefill step fat
(M = batch * prompt). The planner picks, per (M, N, K, epilogue):

* a tile from {64x64, 64x128, 128x128, 128x256, 256x128} sized to M,
* a split-K factor so the grid covers the 256 CUs (cdna_hip_programming.md §5 'Projection
  GEMM at M = 256': choose SPLITK so that tiles * SPLITK ~ 0.5-1x the CU count),
* every GEMM runs on our kernels (no vendor-library backend): decode GEMMs (the hipGraph
  steps) on tiles autotuned at graph capture (on by default; ``DLI_GEMM_AUTOTUNE=0``
  disables it); prefill GEMMs on our 8-phase 256x256 kernel or the one-wave-per-SIMD 256x256
  kernel (tile 45), whichever the warmup measures faster per token bucket
  (``prefill_candidates``).

Split-K partial slabs live in a grow-only per-device workspace; engines warm every shape
up before hipGraph capture so no allocation happens inside a capture.
"""
from __future__ import annotations

import math
import os
import threading
import time
from dataclasses import dataclass

import numpy as np
import torch

# tile id -> (BM, BN); 0-4 stage K through 2 LDS buffers, 5-9 are the same tiles with 3
# buffers and one tile kept in flight across the K-step barrier (gemm.hip)
TILES = {0: (64, 64), 1: (64, 128), 2: (128, 128), 3: (128, 256), 4: (256, 128),
         5: (64, 64), 6: (64, 128), 7: (128, 128), 8: (128, 256), 9: (256, 128),
         10: (192, 128), 11: (192, 128), 12: (160, 128),
         # 8 waves / 512 threads (fewer L2 re-reads of A and W at M >= 256)
         13: (256, 256), 14: (256, 128), 15: (128, 256), 16: (256, 128), 17: (128, 256),
         # grid-filling tiles for N = 6144 / 4096 at M = 512
         18: (128, 96), 19: (128, 96), 20: (128, 64), 21: (128, 64),
         # 256x256 8-phase ping-pong (two wave groups alternate MFMA / load segments)
         22: (256, 256),
         # 192-wide, 8 waves: N = 6144 is 32 column tiles (fused QKV at M = 512 fills the chip
         # with split-K 2 / 4)
         23: (128, 192), 24: (128, 192), 25: (256, 192),
         # 256x224 ping-pong: N = 28672 (Llama-3 gate/up) at M = 512 = 256 tiles on 256 CUs
         26: (256, 224),
         # 256x128 ping-pong: Mixtral grouped down (N = 4096: 32 column tiles per expert),
         # N = 4096 at M = 512 with split-K 4
         28: (256, 128),
         # 256x256, 4 waves (one per SIMD), 128x128 wave tiles, accumulators pinned in the AGPR
         # file (gemm4w_kernel); 41 = 34 with a 3-stage weight ring (160 KiB LDS: W fetched a
         # K-tile further ahead); 45 = 34 with two barriers per K-tile (the buffer released
         # after 20 MFMAs, the next-next K-tile's DMA over 80 MFMAs). The losing A/B variants
         # 35-40 / 42-44 / 46-53 are not instantiated (profiles/r4/gemm4w/)
         34: (256, 256), 41: (256, 256), 45: (256, 256),
         # 55 = 45 persistent: one workgroup per CU walks its tiles, the next tile's first two
         # K-tiles staged in the current tile's last two (gemm4wp.hip); no split-K / grouped
         55: (256, 256)}
# the 4-wave plan raced against the 8-phase one in the prefill autotune
PREFILL_4W_TILE = 45
# the persistent 4-wave tile (55) raced too
PREFILL_PERSIST = True
# prefill-sized grouped expert GEMMs (ops.moe_mlp's eager path): Mixtral 8x7B at 32k routed
# rows, tile 45 vs the 8-phase tile 22: down 2,895 vs 3,071-3,239 us, gate/up 5,736 vs
# 5,898 us (profiles/r4/moe/)
MOE_PREFILL_TILE = 45
# weight-streaming skinny GEMM (gemm.hip gemv_kernel) for M <= GEMV_MAX_M rows: 16 / 32 output
# rows per workgroup (31 for the SiLU*up gate/up pairing); not an MFMA tile, so kept apart
GEMV_TILES = {30: 16, 31: 32, 32: 16, 33: 32,   # 32 / 33: 4 K-steps in flight per lane, M = 1
              29: 16,   # 29: SiLU*up on the 16-row grid (8 gate + 8 up rows), M <= 4
              56: 4, 57: 8,   # 4 / 8 rows a workgroup, 8 K-steps in flight (not SiLU)
              58: 4, 59: 8}   # SiLU*up pairing (2 + 2 / 4 + 4 rows), 8 K-steps in flight
GEMV_M1_ONLY = (32, 33)
GEMV_MAX_M = 4
# batch-1 decode without split-K reduces (ops.linear_residual, ops.NormedRows): the GEMVs that
# add into the residual (epi "res", full K per workgroup) and the tiles whose prologue applies
# a deferred RMSNorm to their input rows (gemv.hip dli_gemv_fused)
GEMV_RES_TILES = {30: 16, 32: 16, 56: 4, 57: 8}
GEMV_PRO_TILES = {"silu_mul": (29, 31, 33, 58, 59), "splitk": (30, 32, 56, 57),
                  "none": (30, 32, 56, 57)}
GEMV_PRO_M1_ONLY = (32, 33)
DEFER_NORM = os.environ.get("DLI_DEFER_NORM", "1") == "1"
TILE_WAVES = {13: (2, 4), 14: (4, 2), 15: (2, 4), 16: (4, 2), 17: (2, 4),
              22: (2, 4), 23: (2, 4), 24: (2, 4), 25: (4, 2),
              26: (4, 2), 28: (4, 2)}


def tile_ok(tile: int, epi: str) -> bool:
    """The SiLU*up epilogue pairs 16-column gate/up blocks inside a wave's column range,
    which must therefore be a multiple of 32."""
    if epi == "res":
        return tile in GEMV_RES_TILES
    if tile in (29, 58, 59):
        return epi == "silu_mul"
    if tile in GEMV_TILES:
        return epi != "silu_mul" or tile in (31, 33)
    if epi != "silu_mul":
        return True
    if tile == 26:              # the straddling gate/up pair meets through LDS
        return True
    bn = TILES[tile][1]
    return (bn // TILE_WAVES.get(tile, (2, 2))[1]) % 32 == 0


# "splitk": a plain GEMM whose fp32 partial slabs feed a fused reduce (ops.linear_add_rmsnorm,
# ops.linear_rope_cache); planned/tuned separately (a non-split winner runs unfused).
EPI = {"none": 0, "f32": 1, "silu_mul": 2, "bias_gelu": 3, "bias": 4, "splitk": 0,
       "slab16": 5}
# tiles whose slab-only split-K call can store fp16 partials (EPI "slab16": the generic tile
# family and the 8-phase kernels); the fused consumers then read half the bytes. The
# weight-streaming GEMVs and the 4-wave family keep fp32 slabs.
SLAB16_TILES = frozenset(list(range(0, 22)) + [22, 23, 24, 25, 26, 28])
SLAB16 = os.environ.get("DLI_SLAB_FP32", "0") != "1"      # A/B: fp32 partials everywhere
# tiles whose grouped SiLU*up GEMM can read its rows through a permutation (the generic
# family: dli_gemm_grouped_gather), so the MoE gate/up skips the gathered copy of its input
GATHER_TILES = frozenset(list(range(0, 22)) + [23, 24, 25])
NUM_CUS = 256


@dataclass(frozen=True)
class GemmPlan:
    backend: str      # "dli": our kernels (the only backend)
    tile: int
    splits: int


_plan_cache: dict = {}
_ws_lock = threading.Lock()
_workspaces: dict = {}
# buffers a larger workspace replaced: a captured hipGraph keeps the pointer it was captured
# with, so a replaced buffer must outlive every graph (the prefill autotune runs after the
# decode graphs are captured and grows the workspace; freeing the old buffer let eager
# tensors take its memory while graph replays still wrote split-K slabs into it)
_retired: list = []


def workspace(device: torch.device, nbytes: int) -> torch.Tensor:
    """Grow-only scratch (bytes) per device. Never freed: see ``_retired``."""
    key = (device.type, device.index)
    with _ws_lock:
        ws = _workspaces.get(key)
        if ws is None or ws.numel() < nbytes:
            if ws is not None:
                _retired.append(ws)
            ws = torch.empty(max(nbytes, 1 << 20), dtype=torch.uint8, device=device)
            _workspaces[key] = ws
        return ws


LARGE_M = 1024


def _heuristic(M: int, N: int, K: int, epi: str) -> GemmPlan:
    """Fitted to profiles/r1_gemm/gemm_bench.json and profiles/r1_gemm8p/ (MI355X, random
    bf16 operands): skinny decode GEMMs (M <= 512) on the 2/3-stage tiles below (autotuned
    at capture); fat prefill GEMMs (M >= LARGE_M) on the 256x256 8-phase ping-pong kernel
    (tile 22) with its fused epilogue (SiLU*up, bias+GELU, fp32); the prefill autotune
    (``prefill_candidates``) may pin the 4-wave tile instead."""
    # M > 512: mixed prefill+decode steps of a full batch and prefill — 256x256 8-phase
    # tiles (the 128-row tiles below ran a 512 + 300-token mixed step's GEMMs ~2.5x slower
    # than the tuned decode step: 26.7 ms per mixed step end to end, profiles/r3/e2e/)
    if M >= LARGE_M or M > 512:
        # mid-sized steps (serving refills / mixed steps of ~1-2k rows): 256x256 tiles leave
        # most CUs idle on the N = 4096 / 6144 projections (M = 1200: 80 / 120 tiles), so
        # split K while the grid stays within one wave of the chip
        tiles = -(-M // 256) * -(-N // 256)
        splits = 1
        if epi in ("none", "splitk"):
            while (tiles * splits * 2 <= NUM_CUS and K % (64 * splits * 2) == 0
                   and K // (splits * 2) >= 1024 and splits < 4):
                splits *= 2
        return GemmPlan("dli", 22, splits)
    if epi == "res":
        # residual-adding GEMV (full K): 4 rows a workgroup, 8 K-steps in flight per lane
        # (1024 workgroups on a 4096-wide projection)
        return GemmPlan("dli", 56, 1)
    if M <= GEMV_MAX_M:
        # batch-1 / tiny batches: stream the weights (gemv_kernel) with enough workgroups
        # (>= 512, two per CU) to keep ~64 KB of loads in flight per CU
        # gate/up at M <= 2: the 16-row SiLU grid (tile 29) 39.5 / 43.3 vs 49.0 / 51.0 us for
        # the 32-row tile 31 at M = 1 / 2 (profiles/r4/b1/s37_*, s38_gemv_sweep_m2.jsonl)
        tile = (29 if M <= 2 else 31) if epi == "silu_mul" else 30
        wgs = -(-N // GEMV_TILES[tile])
        splits = 1
        while (wgs * splits < 512 and K % (64 * splits * 2) == 0
               and K // (splits * 2) >= 1024 and splits < 8):
            splits *= 2
        if epi == "splitk" and splits == 1 and K % 128 == 0:
            splits = 2
        return GemmPlan("dli", tile, splits)
    if M <= 128:
        tile = 0 if N <= 8192 else 1
    elif M <= 256:
        tile = 1 if N <= 8192 else 2
    else:
        tile = 2
    bm, bn = TILES[tile]
    tiles = -(-M // bm) * -(-N // bn)
    splits = 1
    # split K until the grid is ~2-3 waves over the 256 CUs, keeping >= 512 K per slice
    while (tiles * splits * 2 <= 3 * NUM_CUS and K % (64 * splits * 2) == 0
           and K // (splits * 2) >= 512 and splits < 8):
        splits *= 2
    if epi == "splitk" and splits == 1 and K % 128 == 0 and K >= 1024:
        splits = 2            # the fused reduce consumes partial slabs: need >= 2 slices
    return GemmPlan("dli", tile, splits)


def grouped_tile(rows: int, groups: int) -> int:
    """Default tile for the grouped (MoE) GEMM over `rows` permuted rows in `groups` experts
    (autotune_grouped() replaces it at graph capture). Each expert's weights should be
    streamed ONCE, so the tile should cover one expert's rows (mean rows = rows / groups,
    plus headroom for routing imbalance) without doubling the MFMA work. Measured on
    Mixtral 8x7B at batch 512 (~128 rows per expert): 128-row tiles 8.5k tok/s (a second
    pass over most experts' weights), 160x128 14.4k, 192x128 10.2k, 256x128 4.8k, 3-stage
    variants slower (1 workgroup per CU)."""
    forced = os.environ.get("DLI_MOE_TILE")
    if forced:
        return int(forced)
    need = 1.25 * rows / max(1, groups)          # mean rows per expert + imbalance headroom
    for bm, tile in ((64, 1), (128, 2), (160, 12), (192, 10)):
        if need <= bm:
            return tile
    return 4              # 256 x 128


_grouped_cache: dict = {}


def grouped_plan(rows: int, N: int, K: int, epi: str, groups: int) -> GemmPlan:
    p = _grouped_cache.get((_bucket(rows), N, K, epi, groups))
    return p if p is not None else GemmPlan("dli", grouped_tile(rows, groups), 1)


def autotune_grouped(rows: int, w: torch.Tensor, epi: str, iters: int = 5, log=None):
    """Pick the grouped-GEMM tile for `rows` permuted rows over the experts of `w`
    ([E, N, K]) with a random routing (what a decode step of rows/top_k tokens sees). The
    expert weights together exceed the Infinity Cache, so every call is cold."""
    from .. import ops
    E, N, K = w.shape
    key = (_bucket(rows), N, K, epi, E)
    if key in _grouped_cache or os.environ.get("DLI_MOE_TILE"):
        return _grouped_cache.get(key)
    dev = w.device
    # per-expert rows of a RANDOM routing (seeded multinomial), not an exactly even split: with
    # 1024 rows over 8 experts an even split fits 128-row tiles exactly, while in situ about
    # half the experts get more than 128 rows and take a second tile pass over their weights
    # (Mixtral b512: the even-split pick ran 13.6k tok/s, the 160-row tile 15.3k)
    counts = np.random.default_rng(1234).multinomial(rows, [1.0 / E] * E).tolist()
    off = torch.tensor([0] + list(__import__("itertools").accumulate(counts)),
                       dtype=torch.int32, device=dev)
    x = (torch.randn(max(rows, 1), K, device=dev) * 0.5).to(w.dtype)
    # the down projection's split plans on the fp16-slab tiles run fused with the combine
    # (ops.moe_down_combine): time them that way (one pick per row, weight 1)
    ones = torch.ones(max(rows, 1), 1, dtype=torch.float32, device=dev)
    ident = torch.arange(max(rows, 1), dtype=torch.int32, device=dev).view(-1, 1)
    comb = torch.empty(max(rows, 1), N, dtype=w.dtype, device=dev)
    best = None
    cands = []
    for tile in sorted(TILES):
        if TILES[tile][0] > 2 * max(64, rows // E + 32) or not tile_ok(tile, epi):
            continue                                  # far taller than an expert's rows
        for splits in (1, 2, 4):                      # split-K for long-K expert GEMMs
            if splits == 1 or (K % (64 * splits) == 0 and K // splits >= 2048):
                cands.append(GemmPlan("dli", tile, splits))
    for p in cands:
        fused = epi == "none" and ops.moe_slab_plan(p)

        def run(p=p, fused=fused):
            if fused:
                ops.moe_down_combine(x, w, off, rows, p, ones, ident, comb)
            else:
                ops._gemm_native(x, w, epi, plan=p, groups=E, group_off=off,
                                 rows_per_group=rows)
        try:
            ms = ops.benchmark(run, iters=iters, warmup=1, graph=_GRAPH_TUNE)
        except Exception:  # noqa: BLE001
            continue
        if best is None or ms < best[1]:
            best = (p, ms)
    if best is not None:
        _grouped_cache[key] = best[0]
        if log:
            log(f"[gemm autotune] grouped rows={rows} E={E} N={N} K={K} {epi}: {best[0]} "
                f"{best[1]*1e3:.1f} us")
    return best


def _bucket(M: int) -> int:
    """Plan-cache key for M: exact up to 512 rows (decode graph buckets are a fixed small
    set and their best plans differ: one plan per power of two let M=320's plan run M=512),
    a multiple of 128 up to 1024 (the sizes of mixed prefill+decode steps of a full batch,
    tuned as a few buckets when serving: StageRunner.autotune_mixed), power-of-two above
    (prefill)."""
    if M <= 512:
        return M
    if M <= 1024:
        return -(-M // 128) * 128
    b = 1
    while b < M:
        b <<= 1
    return b


def plan(M: int, N: int, K: int, epi: str) -> GemmPlan:
    key = (_bucket(M), N, K, epi)
    p = _plan_cache.get(key)
    if p is not None:
        return p
    p = _heuristic(M, N, K, epi)
    _plan_cache[key] = p
    return p


def set_plan(M: int, N: int, K: int, epi: str, p: GemmPlan) -> None:
    _plan_cache[(_bucket(M), N, K, epi)] = p


def clear_plans() -> None:
    _plan_cache.clear()
    _tuned.clear()


def autotune(shapes, weights: dict, device, iters: int = 6, log=None,
             cold_bytes: int = 1 << 30, qkv_heads=None, candidates=None,
             normed_in=()) -> dict:
    """Measure every candidate plan for each (M, N, K, epi) and pin the fastest
    ("measure, don't guess"). ``weights[(N, K)]`` is a real [N, K] weight of that shape.

    Measured the way a decode step sees it: the weight is COLD (each call reads a different
    copy; the copies together exceed the 256 MB Infinity Cache — timing one warm weight
    picked plans that ran 12 % slower in the model), and split-K plans pay their slab
    reduction (a "splitk" GEMM feeds a fused reduce that reads every slab). A non-split
    winner for a "splitk" shape also becomes that shape's plain plan (unfused path).
    ``qkv_heads`` = (hq, hkv, hd): the "splitk" shape with N = (hq + 2 hkv) hd is the fused
    QKV projection, whose consumer is the decode attention prologue (slab sum or bf16 read,
    RoPE, KV write), so its candidates are timed with the RoPE + cache-write kernel of the
    same input (``ops.linear_rope_cache``) instead of the add + RMSNorm one.
    ``candidates(M, N, K, epi)`` replaces the plan list (``prefill_candidates``).
    ``normed_in``: (N, K, epi) of the GEMMs whose input at M <= GEMV_MAX_M is a deferred
    RMSNorm (``ops.NormedRows``: the batch-1 QKV and gate/up), timed with that prologue.
    Returns {shape: (plan, ms)}."""
    from .. import ops  # local import: ops imports this module
    out = {}
    for (M, N, K, epi) in shapes:
        key = (_bucket(M), N, K, epi)
        if key in _tuned:
            continue
        w0 = weights[(N, K)]
        n_copies = max(2, min(16, -(-cold_bytes // (w0.numel() * w0.element_size()))))
        ws_ = [w0] + [w0.clone() for _ in range(n_copies - 1)]
        x = (torch.randn(M, K, device=device) * 0.5).to(w0.dtype)
        x_in = x
        if M <= GEMV_MAX_M and (N, K, epi) in normed_in:
            x_in = ops.NormedRows(x, torch.ones(K, dtype=w0.dtype, device=device), 1e-5)
        is_qkv = (epi == "splitk" and qkv_heads is not None
                  and N == (qkv_heads[0] + 2 * qkv_heads[1]) * qkv_heads[2])
        if epi == "splitk":
            # a "splitk" GEMM is timed WITH its consumer: split plans reduce their slabs in a
            # fused add+RMSNorm, unsplit plans write bf16 and run the separate add+RMSNorm
            # pass; timing the unsplit GEMM alone hid that pass and biased the choice
            res = torch.zeros(M, N, dtype=w0.dtype, device=device)
            nw = torch.ones(N, dtype=w0.dtype, device=device)
        if epi == "res":
            res_r = torch.zeros(M, N, dtype=w0.dtype, device=device)
        if is_qkv:
            from . import reference as R
            hq, hkv, hd = qkv_heads
            pos = torch.zeros(M, dtype=torch.int32, device=device)
            slots = torch.arange(M, dtype=torch.int32, device=device)
            kc = torch.empty(-(-M // 16), hkv, 16, hd, dtype=w0.dtype, device=device)
            vc = torch.empty_like(kc)
            cs = R.rope_cos_sin(16, hd, 10000.0, device=device)
            # decode-sized QKV: its consumer is the fused reduce + RoPE + KV write + attention
            # kernel where the plan's split count allows it (ops.linear_rope_attention), else
            # the RoPE/cache kernel + attention; time each plan with the path it will run
            # (one-token contexts: the launch and dependency structure, not the KV stream)
            decode_qkv = M <= 512 and candidates is None
            if decode_qkv:
                bt = (slots // 16).to(torch.int32).unsqueeze(1).contiguous()
                ctx = torch.ones(M, dtype=torch.int32, device=device)
                sc = 1.0 / math.sqrt(hd)
        best = None
        timed = []                                  # (ms, plan, run) of every valid candidate
        t_shape = time.perf_counter()
        for p in (candidates or candidate_plans)(M, N, K, epi):
            def run(p=p):
                for w in ws_:
                    if is_qkv and decode_qkv:
                        _qkv_decode(ops, x_in, w, p, pos, slots, cs, kc, vc, bt, ctx, hq, hkv,
                                    hd, sc)
                    elif x_in is not x:
                        ops.linear_normed(x_in, w, epi, plan=p)
                    elif is_qkv:
                        ops.linear_rope_cache(x, w, pos, slots, cs, kc, vc, hq, hkv, hd,
                                              plan=p)
                    elif epi == "splitk":
                        ops.linear_add_rmsnorm(x, w, res, nw, 1e-5, plan=p)
                    elif epi == "res":
                        ops.linear_residual(x, w, res_r, plan=p)
                    else:
                        ops._gemm_native(x, w, epi, plan=p)
            try:
                ms = ops.benchmark(run, iters=iters, warmup=1, graph=_GRAPH_TUNE) / len(ws_)
            except Exception:  # noqa: BLE001 — an invalid candidate is skipped
                continue
            timed.append((ms, p, run))
        best = _final_round(ops, timed, iters, len(ws_))
        del ws_, timed
        if best is not None:
            _plan_cache[key] = best[0]
            _tuned.add(key)
            if epi == "splitk" and best[0].splits == 1:
                _plan_cache[(_bucket(M), N, K, "none")] = best[0]
                _tuned.add((_bucket(M), N, K, "none"))
            out[(M, N, K, epi)] = best
            if log:
                log(f"[gemm autotune] M={M} N={N} K={K} {epi}: {best[0]} {best[1]*1e3:.1f} us "
                    f"({time.perf_counter() - t_shape:.1f} s)")
    return out


# finalists re-timed round-robin after the first pass: candidates within FINAL_BAND of the
# fastest, at most FINAL_N of them, FINAL_ROUNDS rounds; the lowest median wins. One pass in
# candidate order let drift and noise pick among plans a few % apart: two runs of the same
# tree on one box pinned different QKV plans (128x192 split 2 vs 128x96 unsplit,
# profiles/r4/prof vs profiles/r5/s06 wave summaries)
FINAL_BAND = 0.06
FINAL_N = 4
FINAL_ROUNDS = 3


def _final_round(ops, timed, iters: int, n_copies: int):
    """(plan, ms) of the winner among ``timed`` = [(ms, plan, run)] (None if empty)."""
    if not timed:
        return None
    timed.sort(key=lambda t: t[0])
    fin = [t for t in timed if t[0] <= timed[0][0] * (1 + FINAL_BAND)][:max(1, FINAL_N)]
    if len(fin) == 1 or FINAL_ROUNDS <= 0:
        return (fin[0][1], fin[0][0])
    samples = [[ms] for ms, _, _ in fin]
    for _ in range(FINAL_ROUNDS):
        for i, (_, _, run) in enumerate(fin):
            samples[i].append(ops.benchmark(run, iters=iters, warmup=1, graph=_GRAPH_TUNE)
                              / n_copies)
    med = [sorted(s)[len(s) // 2] for s in samples]
    i = min(range(len(fin)), key=lambda j: med[j])
    return (fin[i][1], med[i])


def _qkv_decode(ops, x, w, p, pos, slots, cs, kc, vc, bt, ctx, hq, hkv, hd, scale):
    """One decode step's QKV projection + attention under plan ``p``, as the model runs it
    (models/model.py ``_llama_layers``): the fused kernel when ``p`` allows it, else the
    RoPE/cache kernel and the decode attention."""
    with _forced_plan(x.shape[0], w.shape[0], x.shape[1], p):
        out = ops.linear_rope_attention(x, w, pos, slots, cs, kc, vc, bt, ctx, 1, hq, hkv, hd,
                                        scale)
        if out is None:
            qkv = ops.linear_rope_cache(x, w, pos, slots, cs, kc, vc, hq, hkv, hd, plan=p)
            ops.decode_attention(qkv, kc, vc, bt, ctx, 1, hq, hkv, hd, scale)


class _forced_plan:
    """Pin the plan of one shape for the duration of a timing call (the fused attention path
    reads its plan from the cache, not from an argument): the "splitk" entry, and for an
    unsplit plan also the "none" entry its plain GEMM takes."""

    def __init__(self, M, N, K, p):
        b = _bucket(M)
        self.keys = [(b, N, K, "splitk")] + ([(b, N, K, "none")] if p.splits == 1 else [])
        self.p = p

    def __enter__(self):
        self.old = [_plan_cache.get(k) for k in self.keys]
        for k in self.keys:
            _plan_cache[k] = self.p

    def __exit__(self, *exc):
        for k, o in zip(self.keys, self.old):
            if o is None:
                _plan_cache.pop(k, None)
            else:
                _plan_cache[k] = o


_tuned: set = set()
# candidates timed as graph replays (ops.benchmark graph=True)
_GRAPH_TUNE = True


def prefill_candidates(M: int, N: int, K: int, epi: str):
    """Prefill-sized GEMMs (M > 1024 rows): our 8-phase 256x256 kernel with the heuristic's
    split count against our one-wave-per-SIMD 256x256 kernel (PREFILL_4W_TILE, the
    two-barrier schedule) at the same split, 1-4 % apart on the square / QKV / gate-up /
    down prefill shapes (profiles/r4/gemm4w/), measured per shape and bucket. At these sizes
    the GEMM is MFMA-bound, so the autotuner times them warm (``cold_bytes`` 1)."""
    out = [_heuristic(M, N, K, epi)]
    base = out[0]
    if base.tile == 22 and PREFILL_4W_TILE > 0:
        out.append(GemmPlan("dli", PREFILL_4W_TILE, base.splits))
    if base.tile == 22 and base.splits == 1 and K % 128 == 0 and PREFILL_PERSIST:
        out.append(GemmPlan("dli", 55, 1))
    return out


def candidate_plans(M: int, N: int, K: int, epi: str):
    if epi == "res":
        return [GemmPlan("dli", t, 1) for t in GEMV_RES_TILES
                if M <= GEMV_MAX_M and not (t == 32 and M > 1)]
    out = []
    # tiles kept out of the autotune candidates (DLI_GEMM_EXCLUDE="..." overrides, "" = none).
    # Default: 26 (256x224). It fills all 256 CUs on the gate/up GEMM and wins the isolated
    # autotune (98.8 vs ~106 us), but in the decode step it ran 97.9 vs 99.0 us per call and
    # the bench 0.3-0.7 % lower in three same-box A/B runs (profiles/r2_s2/README.md)
    # 45 stays
    # prefill-only too (no gain in a same-box bench A/B, profiles/r4/bench/s18_*); 41 won
    # isolated decode timings (M = 512 LM head 4-7 %) but cost the step 1.8 % in a same-box
    # bench A/B (42,548 without vs 41,790 / 41,653 tok/s with, profiles/r4/bench/)
    excl_env = os.environ.get("DLI_GEMM_EXCLUDE")
    # 34 too (round 5): the 4-wave family wins isolated cold-weight timings within the noise
    # but loses in the decode graph — down at M = 512 ran 70.4 us on tile 34 against 56.9 on
    # the 8-phase tile 22, the LM head 433 vs 407 (profiles/r5/s12/wave_summary.txt vs
    # profiles/r4/prof/llama_b512_head.wave.txt); the autotune flipped between them run to run
    excl = {int(t) for t in (excl_env if excl_env is not None else "26,34,41,45,55").split(",")
            if t.strip()}
    # ... except where 256x256 tiles take more than one wave of the chip and 256x224 tiles
    # land on a whole number of waves (Llama-3-70B gate/up at M = 512: N = 57344 is 448
    # 256x256 tiles = 1.75 waves, 512 256x224 tiles = 2 waves); an explicit
    # DLI_GEMM_EXCLUDE keeps the list as given
    if excl_env is None and 26 in excl:
        t256 = -(-M // 256) * -(-N // 256)
        t224 = -(-M // 256) * -(-N // 224)
        if t256 > NUM_CUS and t224 % NUM_CUS == 0:
            excl.discard(26)
    for tile, (bm, bn) in TILES.items():
        if not tile_ok(tile, epi) or tile in excl:
            continue
        if M <= 64 and bm > 64:
            continue
        if M > 512 and bm < 128:
            continue
        for splits in (1, 2, 4, 8):
            if K % (64 * splits) or K // splits < 256:
                continue
            tiles = -(-M // bm) * -(-N // bn)
            if splits > 1 and tiles * splits > 4 * NUM_CUS:
                continue
            out.append(GemmPlan("dli", tile, splits))
    if M <= GEMV_MAX_M:
        for tile in GEMV_TILES:
            if tile in excl or not tile_ok(tile, epi) or (tile in GEMV_M1_ONLY and M > 1):
                continue
            for splits in (1, 2, 4, 8):
                if K % (64 * splits) == 0 and K // splits >= 512:
                    out.append(GemmPlan("dli", tile, splits))
    return out
