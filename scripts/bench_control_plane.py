#!/usr/bin/env python3
"""Capacity of the serving control plane alone (no GPU): the master (uvicorn ASGI front,
sqlite store, request queue, async dispatcher) in front of a FAKE worker whose /inference
answers after a fixed engine time with unlimited concurrency, driven by the closed-loop load
generator. With an engine that never saturates, any shortfall of

    requests/s  <  concurrency / engine_s

is latency the master / HTTP / load-generator path adds per request, i.e. what the end-to-end
config-2 run (scripts/serve_e2e.sh) loses before the GPU is even involved.

    python scripts/bench_control_plane.py --concurrency 1024 --requests 4096 --engine-s 0.7
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import subprocess
import sys
import tempfile
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def fake_worker_app(engine_s: float, result: str):
    async def app(scope, receive, send):
        if scope["type"] != "http":
            return
        path = scope["path"]
        body = b""
        while True:
            m = await receive()
            body += m.get("body", b"")
            if not m.get("more_body"):
                break
        if path == "/health":
            out = {"status": "healthy", "resources": {"cpu": 0.0, "memory": 0.0, "gpu": 0.0},
                   "loaded_shards": []}
        elif path == "/inference":
            t0 = time.time()
            await asyncio.sleep(engine_s)
            out = {"status": "success", "result": result, "execution_time": time.time() - t0,
                   "output_tokens": 68, "finish_reason": "length"}
        else:
            out = {"status": "success", "message": "ok"}
        data = json.dumps(out).encode()
        await send({"type": "http.response.start", "status": 200,
                    "headers": [(b"content-type", b"application/json"),
                                (b"content-length", str(len(data)).encode())]})
        await send({"type": "http.response.body", "body": data})
    return app


def serve_fake_worker(port: int, engine_s: float):
    import uvicorn
    uvicorn.run(fake_worker_app(engine_s, "lorem ipsum " * 40), host="127.0.0.1", port=port,
                log_level="warning", backlog=4096)


def wait_http(url: str, timeout: float = 60.0):
    import requests
    t0 = time.time()
    while time.time() - t0 < timeout:
        try:
            if requests.get(url, timeout=2).status_code < 500:
                return True
        except requests.RequestException:
            time.sleep(0.3)
    return False


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--concurrency", type=int, default=1024)
    ap.add_argument("--requests", type=int, default=4096)
    ap.add_argument("--engine-s", type=float, default=0.7)
    ap.add_argument("--master-port", type=int, default=8731)
    ap.add_argument("--worker-port", type=int, default=5731)
    ap.add_argument("--server", default="aiohttp", choices=["uvicorn", "aiohttp"])
    ap.add_argument("--master-procs", type=int, default=1,
                    help="serve-master --procs (aiohttp: processes sharing port + database)")
    ap.add_argument("--profile", default="", help="write a sampling profile of the master")
    ap.add_argument("--fake-worker", action="store_true", help=argparse.SUPPRESS)
    a = ap.parse_args()
    if a.fake_worker:
        serve_fake_worker(a.worker_port, a.engine_s)
        return 0
    import requests
    env = dict(os.environ)
    db = tempfile.mktemp(suffix=".sqlite3", prefix="dli_cp_")
    env.update(MASTER_DB=db, DISPATCH_WORKERS=str(a.concurrency), PYTHONPATH=str(ROOT),
               DLI_LOG_DIR=tempfile.mkdtemp(prefix="dli_cp_logs_"))
    procs = []
    try:
        procs.append(subprocess.Popen([sys.executable, __file__, "--fake-worker",
                                       "--worker-port", str(a.worker_port),
                                       "--engine-s", str(a.engine_s)], env=env))
        mcmd = ["-m", "distributed_llm_inferencing_amd.cli"]
        if a.profile:     # the master under the sampling profiler (scripts/sample_profile.py)
            mcmd = [str(ROOT / "scripts" / "sample_profile.py"), "--out", a.profile,
                    *(["--cprofile"] if a.profile.endswith(".txt") else []),
                    "distributed_llm_inferencing_amd.cli"]
        procs.append(subprocess.Popen([sys.executable, *mcmd,
                                       "serve-master", "--port", str(a.master_port),
                                       "--server", a.server, "--procs", str(a.master_procs)],
                                      env=env,
                                      stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL))
        master = f"http://127.0.0.1:{a.master_port}"
        if not (wait_http(f"http://127.0.0.1:{a.worker_port}/health")
                and wait_http(f"{master}/api/inference/recent/")):
            print(json.dumps({"error": "servers did not come up"}))
            return 1
        r = requests.post(f"{master}/api/nodes/add/",
                          data={"hostname": "fake0", "ip_address": "127.0.0.1",
                                "port": a.worker_port}, timeout=10)
        r.raise_for_status()
        lg = [sys.executable, "-m", "distributed_llm_inferencing_amd.loadgen", "--master", master,
              "--model", "llama3-8b", "--prompt-words", "5"]
        subprocess.run(lg + ["--requests", str(a.concurrency), "--concurrency",
                             str(a.concurrency), "--seed", "99"], env=env, check=True,
                       stdout=subprocess.DEVNULL)
        import psutil
        mp = psutil.Process(procs[1].pid)
        ps = {"fake_worker": [psutil.Process(procs[0].pid)],
              "master": [mp] + mp.children(recursive=True)}

        def cpu_s(k):
            return sum(sum(p.cpu_times()[:2]) for p in ps[k])
        cpu0 = {k: cpu_s(k) for k in ps}
        import resource
        ru0 = resource.getrusage(resource.RUSAGE_CHILDREN)
        t0 = time.time()
        lgp = subprocess.run(lg + ["--requests", str(a.requests), "--concurrency",
                                   str(a.concurrency)], env=env, check=True,
                             capture_output=True, text=True)
        wall = time.time() - t0
        cpu = {k: round((cpu_s(k) - cpu0[k]) / wall, 3) for k in ps}
        ru1 = resource.getrusage(resource.RUSAGE_CHILDREN)
        cpu["loadgen"] = round((ru1.ru_utime + ru1.ru_stime - ru0.ru_utime - ru0.ru_stime)
                               / wall, 3)
        out = lgp.stdout.strip().splitlines()[-1]
        rep = json.loads(out)
        ideal = a.concurrency / a.engine_s
        rep.update(engine_s=a.engine_s, ideal_requests_per_s=round(ideal, 1),
                   control_plane_latency_s=round(a.concurrency / rep["requests_per_s"]
                                                 - a.engine_s, 4)
                   if rep.get("requests_per_s") else None,
                   cpus=os.cpu_count(), cores_busy=cpu, master_server=a.server,
                   master_procs=a.master_procs)
        print(json.dumps(rep), flush=True)
        return 0
    finally:
        for p in procs:
            p.terminate()
        for p in procs:
            try:
                p.wait(10)
            except subprocess.TimeoutExpired:
                p.kill()
        for suffix in ("", "-wal", "-shm"):
            try:
                os.remove(db + suffix)
            except OSError:
                pass


if __name__ == "__main__":
    sys.exit(main())
