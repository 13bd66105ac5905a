#!/usr/bin/env python3
"""Closed-loop simulation of the engine's admission policy (CPU only, no model): the real
``Scheduler`` + C++ ``BlockManager`` stepped against a fake clock whose step costs are fitted
to MI355X measurements, with C clients that resubmit after a control-plane delay.

Step cost model (Llama-3-8B bf16, batch up to 512; profiles/r3/epi_tr, profiles/r3/e2e):
    decode step                      t_dec(rows)  (graph replay; ~flat in rows above 256)
    mixed / prefill step             t_dec(decode rows) + prefill_tokens * t_tok + t_mixed
so a refill costs its prompts' FLOPs plus a fixed overhead (eager launches, larger-M plans).
The end-to-end question it answers: which admission pacing keeps the decode batch full
without paying the mixed-step overhead too often.

    python scripts/sim_admission.py --refill 0.06 --admit-min-frac 0.125
"""
from __future__ import annotations

import argparse
import collections
import json
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))


class FakeClock:
    def __init__(self):
        self.t = 0.0

    def perf_counter(self):
        return self.t

    def time(self):
        return self.t


def t_dec(rows: int, a) -> float:
    return a.t_dec * (0.55 + 0.45 * min(rows, 512) / 512) if rows else 0.0


def run(a) -> dict:
    from distributed_llm_inferencing_amd.engine import scheduler as S
    from distributed_llm_inferencing_amd.engine.sequence import SamplingParams
    from distributed_llm_inferencing_amd.runtime import BlockManager
    clock = FakeClock()
    S.time = clock                                  # the scheduler's pacing reads this clock
    bm = BlockManager(65536, 16)
    sch = S.Scheduler(bm, max_seqs_per_mb=a.max_batch, max_prefill_tokens=16384,
                      max_model_len=2048, eos_token_id=None, mixed_steps=True,
                      prefix_caching=False, admit_window_s=a.admit_window,
                      admit_min_frac=a.admit_min_frac, refill_interval_s=a.refill)
    sp = SamplingParams(max_length=a.prompt + a.gen, ignore_eos=True)
    rng = np.random.default_rng(0)
    pending = collections.deque()                 # (time it reaches the engine, rid)
    nid = [0]

    def submit(at):
        pending.append((at, nid[0]))
        nid[0] += 1
    def delay():                                   # control-plane latency, jittered
        return float(rng.exponential(a.delay_in + a.delay_out))
    for i in range(a.concurrency):
        submit(float(rng.uniform(0, a.ramp)))
    inflight = None
    steps = rows_sum = tokens = mixed = 0
    done = 0
    t_start = None
    while done < a.requests:
        if pending and len(pending) > 1 and pending[-1][0] < pending[-2][0]:
            pending = collections.deque(sorted(pending))
        while pending and pending[0][0] <= clock.t:
            _, rid = pending.popleft()
            seq = sch.add_request(f"r{rid}", rng.integers(1000, 100000, a.prompt).tolist(), sp)
            seq.arrival = clock.t
        meta = sch.schedule(0, inflight=inflight)
        if meta is None and inflight is None:
            clock.t = pending[0][0] if pending else clock.t + 0.001
            continue
        dt = 0.0
        if meta is not None:
            nd = meta.num_decode if meta.kind == 1 else meta.num_seqs
            dt = t_dec(nd, a)
            if meta.kind == 1:
                dt += (meta.num_tokens - meta.num_decode) * a.t_tok + a.t_mixed
                mixed += 1
            steps += 1
            rows_sum += meta.num_seqs
        clock.t += max(dt, 1e-4)
        if inflight is not None:
            sch.update(inflight, np.ones(inflight.num_seqs, dtype=np.int32) * 7)
            tokens += inflight.num_sampled
        inflight = meta
        for seq in sch.pop_finished():
            done += 1
            if done == a.requests // 4:
                t_start, tok0 = clock.t, tokens
            submit(clock.t + delay())
    wall = clock.t - t_start
    return {"refill_s": a.refill, "admit_min_frac": a.admit_min_frac,
            "tok_per_s": round((tokens - tok0) / wall), "rows_per_step": round(rows_sum / steps, 1),
            "mixed_share": round(mixed / steps, 3), "steps": steps}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--concurrency", type=int, default=1024)
    ap.add_argument("--requests", type=int, default=6000)
    ap.add_argument("--max-batch", type=int, default=512)
    ap.add_argument("--prompt", type=int, default=31)
    ap.add_argument("--gen", type=int, default=69)
    ap.add_argument("--t-dec", type=float, default=0.0093)
    ap.add_argument("--t-tok", type=float, default=10e-6)
    ap.add_argument("--t-mixed", type=float, default=0.0045)
    ap.add_argument("--delay-in", type=float, default=0.05, help="client -> engine (s)")
    ap.add_argument("--delay-out", type=float, default=0.03, help="engine -> next submit (s)")
    ap.add_argument("--refill", type=float, default=0.06)
    ap.add_argument("--admit-min-frac", type=float, default=0.125)
    ap.add_argument("--admit-window", type=float, default=0.02)
    ap.add_argument("--ramp", type=float, default=1.0, help="clients start over this many s")
    ap.add_argument("--sweep", action="store_true")
    a = ap.parse_args()
    if not a.sweep:
        print(json.dumps(run(a)))
        return
    for frac in (0.125, 0.03, 0.0):
        for refill in (0.0, 0.015, 0.03, 0.06, 0.12):
            a.refill, a.admit_min_frac = refill, frac
            print(json.dumps(run(a)), flush=True)


if __name__ == "__main__":
    main()
