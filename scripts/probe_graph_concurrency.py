"""Do independent branches of a captured hipGraph run concurrently on this ROCm build?

Two forked capture streams each run one single-workgroup spin kernel (torch.cuda._sleep);
the replay takes ~1x one spin if the branches overlap, ~2x if the graph serialises them.
Eager two-stream timing is printed beside it. One JSON line per mode.
"""
import json
import time

import torch


def main():
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    cyc = 20_000_000                       # ~10 ms at ~2 GHz
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

    def branches():
        # fork from the stream current at call time: inside torch.cuda.graph that is the
        # capture stream (forking from the default stream left the graph empty)
        main_s = torch.cuda.current_stream()
        s1.wait_stream(main_s)
        s2.wait_stream(main_s)
        with torch.cuda.stream(s1):
            torch.cuda._sleep(cyc)
        with torch.cuda.stream(s2):
            torch.cuda._sleep(cyc)
        main_s.wait_stream(s1)
        main_s.wait_stream(s2)

    def timed(fn, n=5):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / n * 1e3

    one = timed(lambda: torch.cuda._sleep(cyc))
    eager = timed(branches)
    g = torch.cuda.CUDAGraph()
    branches()
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        branches()
    graph = timed(g.replay)
    for mode, ms in (("one_spin", one), ("eager_two_streams", eager), ("graph_two_branches", graph)):
        print(json.dumps({"mode": mode, "ms": round(ms, 3), "ratio_to_one": round(ms / one, 3)}))


if __name__ == "__main__":
    main()
