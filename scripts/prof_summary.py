#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace --stats CSV directory: top kernels + GPU busy time."""
import csv
import sys
from pathlib import Path

d = Path(sys.argv[1])
stats = next(d.glob("*kernel_stats.csv"))
rows = list(csv.DictReader(open(stats)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"{'ms':>9} {'%':>5} {'calls':>7} {'avg_us':>8}  kernel")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:int(sys.argv[2]) if len(sys.argv) > 2 else 25]:
    print(f"{float(r['TotalDurationNs'])/1e6:9.2f} {100*float(r['TotalDurationNs'])/tot:5.1f} "
          f"{r['Calls']:>7} {float(r['AverageNs'])/1e3:8.1f}  {r['Name'][:100]}")
print(f"total kernel ms {tot/1e6:.1f}")
tr = list(d.glob("*kernel_trace.csv"))
if tr:
    ev = sorted((int(x["Start_Timestamp"]), int(x["End_Timestamp"])) for x in csv.DictReader(open(tr[0])))
    busy, cur_s, cur_e = 0, None, None
    for s, e in ev:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    span = ev[-1][1] - ev[0][0]
    print(f"trace span {span/1e6:.1f} ms, GPU busy (union) {busy/1e6:.1f} ms = {100*busy/span:.1f}%")
