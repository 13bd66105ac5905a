#!/usr/bin/env python3
"""Merge rocprofv3 --pmc pass directories into one per-kernel counter table.

    pmc_report.py [--tail N] <pass_dir> [<pass_dir> ...]

Every ``*counter_collection.csv`` under the given directories is read; values are averaged
per (kernel, grid size, counter) over the dispatches of that kernel at that grid (one row per
GEMM shape / plan). ``--tail N`` keeps only the last N dispatches of each pass (by
Dispatch_Id): the timed waves of a bench run, without its capture-time autotune probes. Derived columns, where their
inputs were collected (gfx94x formulas, the only ones ROCm 7.2 ships for gfx950):

* mfma_busy%  = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / XCDs * CUs * 4 SIMDs).
  On gfx950 GRBM_GUI_ACTIVE is summed over the 8 XCCs (it reads ~8x the kernel's cycles)
  and the MFMA busy count is per SIMD; with that normalisation the 8-phase gate/up GEMM
  reads 49 %, matching its analytic 1.17 PF/s of the 2.5 PF/s dense bf16 peak.
* mfma_GF     = SQ_INSTS_VALU_MFMA_MOPS_BF16 * 512 / 1e9 (GFLOP per call; 1 MOP = 512 FLOPs on gfx950)
* ea_rd_MB    = 32*RDREQ_32B + 64*RDREQ_64B + 128*RDREQ_128B (L2 -> fabric read bytes).
  The shipped FETCH_SIZE expression counts 128-byte requests via TCC_BUBBLE; both are
  reported so the gap is visible.
* lds_conf%   = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
* hbm_rd_MB   = FETCH_SIZE (KB) / 1024,   hbm_wr_MB = WRITE_SIZE (KB) / 1024
* wait/issue/active% = SQ_WAIT_ANY / SQ_WAIT_INST_ANY / SQ_ACTIVE_INST_ANY over SQ_WAVE_CYCLES
"""
import csv
import sys
from collections import defaultdict
from pathlib import Path

CUS = 256
XCDS = 8
SIMDS = 4


def short(name: str) -> str:
    n = name.split("(")[0]
    return n.replace("void ", "")[:44]


def main():
    args = sys.argv[1:]
    tail = 0
    if len(args) >= 2 and args[0] == "--tail":
        tail, args = int(args[1]), args[2:]
    vals = defaultdict(lambda: defaultdict(list))
    for d in args:
        for f in Path(d).rglob("*counter_collection.csv"):
            rows = list(csv.DictReader(open(f)))
            if tail:
                ids = sorted({int(r.get("Dispatch_Id", 0) or 0) for r in rows})
                cut = ids[-tail] if len(ids) >= tail else ids[0] if ids else 0
                rows = [r for r in rows if int(r.get("Dispatch_Id", 0) or 0) >= cut]
            for r in rows:
                k = short(r.get("Kernel_Name", "?"))
                g = r.get("Grid_Size")
                if g:
                    k = f"{k} g={g}"
                try:
                    # one row per (dispatch, counter); averaged per call below
                    vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
                except (KeyError, ValueError):
                    continue
    if not vals:
        print("no counter_collection.csv found")
        return
    counters = sorted({c for v in vals.values() for c in v})
    print("per-dispatch means")
    for k in sorted(vals):
        m = {c: sum(x) / len(x) for c, x in vals[k].items()}
        calls = max(len(x) for x in vals[k].values())
        line = [f"{k:58s} n={calls:5d}"]
        gui = m.get("GRBM_GUI_ACTIVE")
        if gui and "SQ_VALU_MFMA_BUSY_CYCLES" in m:
            line.append(f"mfma_busy%="
                        f"{100 * m['SQ_VALU_MFMA_BUSY_CYCLES'] / (gui / XCDS * CUS * SIMDS):5.1f}")
        if "SQ_INSTS_VALU_MFMA_MOPS_BF16" in m:
            line.append(f"mfma_GF={m['SQ_INSTS_VALU_MFMA_MOPS_BF16'] * 512 / 1e9:8.2f}")
        if m.get("SQ_LDS_IDX_ACTIVE") and "SQ_LDS_BANK_CONFLICT" in m:
            line.append(f"lds_conf%={100 * m['SQ_LDS_BANK_CONFLICT'] / m['SQ_LDS_IDX_ACTIVE']:5.1f}")
        if "FETCH_SIZE" in m:
            line.append(f"hbm_rd_MB={m['FETCH_SIZE'] / 1024:8.1f}")
        rq = [m.get(f"TCC_EA0_RDREQ_{b}B_sum") for b in (32, 64, 128)]
        if all(v is not None for v in rq):
            line.append(f"ea_rd_MB={(32 * rq[0] + 64 * rq[1] + 128 * rq[2]) / 2**20:8.1f}")
        if "TCC_EA0_RDREQ_DRAM_sum" in m and "TCC_EA0_RDREQ_sum" in m and m["TCC_EA0_RDREQ_sum"]:
            line.append(f"dram_req%={100 * m['TCC_EA0_RDREQ_DRAM_sum'] / m['TCC_EA0_RDREQ_sum']:5.1f}")
        if "WRITE_SIZE" in m:
            line.append(f"hbm_wr_MB={m['WRITE_SIZE'] / 1024:8.1f}")
        wc = m.get("SQ_WAVE_CYCLES")
        if wc:
            parts = [(n, m.get(c)) for n, c in (("wait", "SQ_WAIT_ANY"),
                                                 ("issue", "SQ_WAIT_INST_ANY"),
                                                 ("active", "SQ_ACTIVE_INST_ANY"))]
            line.append(" ".join(f"{n}%={100 * v / wc:4.1f}" for n, v in parts if v is not None))
        print("  ".join(line))
    print("\nraw counters (per-dispatch mean)")
    print("kernel," + ",".join(counters))
    for k in sorted(vals):
        row = [k]
        for c in counters:
            x = vals[k].get(c)
            row.append(f"{sum(x) / len(x):.4g}" if x else "")
        print(",".join(row))


if __name__ == "__main__":
    main()
