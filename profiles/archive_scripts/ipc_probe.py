"""Same-GPU multi-process probe of the hipIpc mailbox transport (csrc/runtime/ipc.cpp).

Run: python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \
         scripts/ipc_probe.py [--flags device|host] [--out FILE]
Every rank computes on cuda:0 (one-GPU box) or cuda:LOCAL_RANK (--per-rank-device). Checks,
in order, each printed as one JSON line by rank 0:
  open      hipIpcOpenMemHandle of a peer allocation on the same device
  fifo      200 ping-pong messages of random sizes, every byte checked
  latency   round trip of an 8 KB message (host-timed over 500 round trips)
  bandwidth one-way 4 MB / 64 MB messages
  graph     the exchange captured in a hipGraph with a kernel on each side, replayed
  abort     (host flags) a receive whose peer never sends, released by abort()
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from datetime import timedelta

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--flags", default="device", choices=["device", "host"])
    ap.add_argument("--per-rank-device", action="store_true")
    ap.add_argument("--skip-graph", action="store_true")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    dist.init_process_group("gloo", timeout=timedelta(seconds=120))
    rank, world = dist.get_rank(), dist.get_world_size()
    dev = torch.device("cuda", int(os.environ.get("LOCAL_RANK", 0)) if a.per_rank_device else 0)
    torch.cuda.set_device(dev)
    from distributed_llm_inferencing_amd.runtime import IpcEndpoint
    results = []

    def report(name, **kw):
        if rank == 0:
            rec = {"check": name, "flags": a.flags,
                   "copy": os.environ.get("DLI_IPC_COPY", "kernel"), **kw}
            print(json.dumps(rec), flush=True)
            results.append(rec)

    big = 64 << 20
    m = [[0 if s == d else big for d in range(world)] for s in range(world)]
    prefix = f"/dli_ipc_probe_{os.environ.get('MASTER_PORT', '0')}" if a.flags == "host" else ""
    ep = IpcEndpoint(world, rank, m, host_prefix=prefix)
    hs = [None] * world
    dist.all_gather_object(hs, ep.handles())
    dist.barrier()
    ep.connect(hs)
    dist.barrier()
    report("open", ok=True)
    s = torch.cuda.current_stream(dev).cuda_stream
    nxt, prv = (rank + 1) % world, (rank - 1) % world

    # FIFO: every rank sends to next, receives from prev, random sizes (same seed everywhere)
    g = torch.Generator().manual_seed(7)
    sizes = torch.randint(1, 1 << 18, (200,), generator=g).tolist()
    bad = 0
    rx = torch.empty(1 << 18, dtype=torch.int32, device=dev)
    for i, n in enumerate(sizes):
        tx = torch.arange(n, dtype=torch.int32, device=dev) * (rank + 1) + i
        ep.exchange([(tx, nxt)], [(rx[:n], prv)], s)
        exp = torch.arange(n, dtype=torch.int32, device=dev) * (prv + 1) + i
        bad += int((rx[:n] != exp).sum().item())
    torch.cuda.synchronize(dev)
    report("fifo", messages=len(sizes), bad_words=bad, ok=bad == 0)

    # latency: rank 0 <-> rank 1 ping-pong, 8 KB
    def pingpong(nbytes, iters):
        t = torch.ones(nbytes // 4, dtype=torch.int32, device=dev)
        r = torch.empty_like(t)
        dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(iters):
            if rank == 0:
                ep.exchange([(t, 1)], [], s)
                ep.exchange([], [(r, 1)], s)
            elif rank == 1:
                ep.exchange([], [(r, 0)], s)
                ep.exchange([(r, 0)], [], s)
        torch.cuda.synchronize(dev)
        return time.perf_counter() - t0

    pingpong(8192, 20)
    dt = pingpong(8192, 500)
    report("latency", bytes=8192, round_trip_us=round(dt / 500 * 1e6, 2))

    for nb in (4 << 20, 64 << 20):
        t = torch.ones(nb // 2, dtype=torch.bfloat16, device=dev)
        r = torch.empty_like(t)
        it = 50 if nb <= (4 << 20) else 20
        dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(it):
            ep.exchange([(t, nxt)], [(r, prv)], s)
        torch.cuda.synchronize(dev)
        dt = time.perf_counter() - t0
        dist.barrier()
        report("bandwidth", bytes=nb, us_per_msg=round(dt / it * 1e6, 1),
               gb_s=round(nb * it / dt / 1e9, 1))

    if not a.skip_graph:
        x = torch.zeros(1024, dtype=torch.float32, device=dev)
        y = torch.zeros(1024, dtype=torch.float32, device=dev)
        gr = torch.cuda.CUDAGraph()
        ok, err = True, ""
        try:
            side = torch.cuda.Stream(dev)
            side.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(side):
                with torch.cuda.graph(gr, stream=side):
                    x.add_(1.0)
                    ep.exchange([(x, nxt)], [(y, prv)], side.cuda_stream)
                    y.mul_(2.0)
            torch.cuda.current_stream(dev).wait_stream(side)
        except Exception as e:  # noqa: BLE001
            ok, err = False, repr(e)[:300]
        okl = [None] * world
        dist.all_gather_object(okl, ok)
        if all(okl):
            vals = []
            for it in range(5):
                gr.replay()
                torch.cuda.synchronize(dev)
                vals.append(float(y[0].item()))
            exp = [2.0 * (it + 1) for it in range(5)]
            report("graph", captured=True, values=vals, expected=exp, ok=vals == exp)
        else:
            report("graph", captured=False, error=err, ok=False)
        dist.barrier()

    if world >= 2:
        # rank 0 waits on a message rank 1 never sends; the host sees nothing pending, aborts
        r = torch.empty(16, dtype=torch.int32, device=dev)
        if rank == 0:
            before = ep.pending(1)
            ep.exchange([], [(r, 1)], s)
            ev = torch.cuda.Event()
            ev.record()
            time.sleep(1.0)
            stuck = not ev.query()
            t0 = time.perf_counter()
            err = None
            while not ev.query() and time.perf_counter() - t0 < 10:
                try:
                    ep.abort(timeout_s=2.0)
                except RuntimeError as e:
                    err = str(e)
                    break
                time.sleep(0.01)
            report("abort", pending_before=before, stuck_before_abort=stuck,
                   released=ev.query(), error=err, ok=stuck and ev.query())
        dist.barrier()
    torch.cuda.synchronize(dev)
    dist.barrier()
    st = ep.stats()
    ep.close()
    report("done", stats=st)
    if rank == 0 and a.out:
        with open(a.out, "w") as f:
            for rec in results:
                f.write(json.dumps(rec) + "\n")
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
