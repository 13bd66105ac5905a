#!/usr/bin/env python3
"""Poor man's sampling profiler for a multi-threaded Python server (py-spy is not installed):
runs a module's ``main`` in this process while a sampler thread reads
``sys._current_frames()`` every --interval seconds and counts, per thread name, the
innermost frames and the inclusive (anywhere-on-stack) functions. On SIGTERM/SIGINT (or
after --duration) it writes the top entries as JSON to --out and exits.

    python scripts/sample_profile.py --out /tmp/master_prof.json -- \\
        distributed_llm_inferencing_amd.cli serve-master --port 8000 --server uvicorn
"""
from __future__ import annotations

import argparse
import collections
import json
import os
import runpy
import signal
import sys
import threading
import time


# innermost frames of a thread that is parked (waiting for work, I/O or a lock)
IDLE = ("threading.py:wait", "selectors.py:select", "thread.py:_worker:81", "store.py:_run:138",
        "queue.py:get", "base_events.py:_run_once")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--interval", type=float, default=0.002)
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--cprofile", action="store_true",
                    help="deterministic cProfile of every thread instead of sampling")
    ap.add_argument("module")
    ap.add_argument("args", nargs=argparse.REMAINDER)
    a = ap.parse_args()
    own = collections.Counter()
    incl = collections.Counter()
    samples = [0]
    stop = threading.Event()
    me = threading.get_ident()

    def key(f):
        c = f.f_code
        return f"{os.path.basename(c.co_filename)}:{c.co_name}:{f.f_lineno}"

    def sampler():
        names = {}
        while not stop.wait(a.interval):
            for t in threading.enumerate():
                names[t.ident] = t.name
            for tid, f in sys._current_frames().items():
                if tid == threading.get_ident():
                    continue
                tn = names.get(tid, "?")
                k0 = key(f)
                own[(tn, k0)] += 1
                if any(k0.startswith(x) for x in IDLE):
                    continue                      # parked thread: no inclusive count
                seen = set()
                while f is not None:
                    k = key(f)
                    if k not in seen:
                        incl[k] += 1
                        seen.add(k)
                    f = f.f_back
            samples[0] += 1

    def dump(*_):
        stop.set()
        res = {"samples": samples[0], "interval_s": a.interval,
               "own": [[t, k, n] for (t, k), n in own.most_common(a.top * 50)],
               "inclusive_busy": [[k, n] for k, n in incl.most_common(a.top * 4)]}
        with open(a.out, "w") as fh:
            json.dump(res, fh, indent=1)
        os._exit(0)

    if a.cprofile:
        # deterministic profile of EVERY thread: a cProfile.Profile per thread, enabled by the
        # threading.setprofile hook on the thread's first event (and here for the main one)
        import cProfile
        import pstats
        profs = []

        def hook(*_):
            p = cProfile.Profile()
            profs.append(p)
            p.enable()

        threading.setprofile(hook)
        main_p = cProfile.Profile()
        profs.append(main_p)

        def dump(*_):                                   # noqa: F811
            for p in profs:
                try:
                    p.disable()
                except Exception:  # noqa: BLE001
                    pass
            st = None
            for p in profs:
                try:
                    p.create_stats()
                    st = pstats.Stats(p) if st is None else st.add(p)
                except Exception:  # noqa: BLE001
                    pass
            with open(a.out, "w") as fh:
                st.stream = fh
                st.sort_stats("tottime").print_stats(a.top * 2)
                st.sort_stats("cumulative").print_stats(a.top * 2)
            os._exit(0)
        main_p.enable()
    signal.signal(signal.SIGTERM, dump)
    signal.signal(signal.SIGINT, dump)
    if not a.cprofile:
        threading.Thread(target=sampler, daemon=True, name="sampler").start()
    sys.argv = [a.module] + [x for x in a.args if x != "--"]
    try:
        runpy.run_module(a.module, run_name="__main__")
    finally:
        dump()


if __name__ == "__main__":
    main()
