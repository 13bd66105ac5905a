#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace --stats CSV directory: top kernels + GPU busy time.

    prof_summary.py <dir> [top_n] [--tail-ms T]

--tail-ms T restricts everything to kernels that started in the last T ms of the trace
(e.g. the timed wave of bench.py, excluding autotune and graph-capture warmup), computed
from the kernel trace instead of the stats file."""
import argparse
import csv
from collections import defaultdict
from pathlib import Path

ap = argparse.ArgumentParser()
ap.add_argument("dir")
ap.add_argument("top", nargs="?", type=int, default=25)
ap.add_argument("--tail-ms", type=float, default=None)
ap.add_argument("--merge", action="store_true",
                help="merge every kernel_trace.csv under the directory (all ranks' processes)")
ap.add_argument("--gaps", type=int, default=0,
                help="also list the N longest GPU-idle gaps (kernel before -> kernel after)")
a = ap.parse_args()
d = Path(a.dir)
tr = sorted(d.rglob("*kernel_trace.csv"))
ev = []
if tr:
    # every process's trace (a same-GPU multi-rank rehearsal writes one per rank): the
    # union is what the one GPU did
    ev = sorted((int(x["Start_Timestamp"]), int(x["End_Timestamp"]), x["Kernel_Name"])
                for f in (tr if a.merge else tr[:1]) for x in csv.DictReader(open(f)))
if a.tail_ms is not None and ev:
    t_end = ev[-1][1]
    ev = [e for e in ev if e[0] >= t_end - a.tail_ms * 1e6]
    agg = defaultdict(lambda: [0, 0])
    for s, e, n in ev:
        agg[n][0] += e - s
        agg[n][1] += 1
    rows = [{"Name": n, "TotalDurationNs": v[0], "Calls": v[1], "AverageNs": v[0] / v[1]}
            for n, v in agg.items()]
else:
    stats = next(d.rglob("*kernel_stats.csv"))
    rows = list(csv.DictReader(open(stats)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"{'ms':>9} {'%':>5} {'calls':>7} {'avg_us':>8}  kernel")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:a.top]:
    print(f"{float(r['TotalDurationNs'])/1e6:9.2f} {100*float(r['TotalDurationNs'])/tot:5.1f} "
          f"{r['Calls']:>7} {float(r['AverageNs'])/1e3:8.1f}  {r['Name'][:100]}")
print(f"total kernel ms {tot/1e6:.1f}")
if ev:
    busy, cur_s, cur_e = 0, None, None
    for s, e, _ in ev:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    span = ev[-1][1] - ev[0][0]
    print(f"trace span {span/1e6:.1f} ms, GPU busy (union) {busy/1e6:.1f} ms = {100*busy/span:.1f}%")
    if a.gaps:
        gaps, end, prev = [], ev[0][1], ev[0][2]
        t0 = ev[0][0]
        for s_, e_, n_ in ev[1:]:
            if s_ > end:
                gaps.append((s_ - end, prev, n_, end - t0))
            if e_ > end:
                end, prev = e_, n_
        gaps.sort(reverse=True)
        idle = sum(g[0] for g in gaps)
        print(f"idle gaps: {len(gaps)}, total {idle/1e6:.2f} ms; "
              f"> 100 us: {sum(1 for g in gaps if g[0] > 1e5)} "
              f"({sum(g[0] for g in gaps if g[0] > 1e5)/1e6:.2f} ms)")
        for g, before, after, at in gaps[:a.gaps]:
            print(f"  {g/1e3:9.1f} us at {at/1e6:8.2f} ms  after {before[:44]}  before {after[:44]}")
