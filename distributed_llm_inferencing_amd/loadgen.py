"""End-to-end load generator for the serving stack (SURVEY.md §7.1 "bench/ load generator":
tokens/s + p50/p99 through the master's public API).

Submits requests to a running master (``POST /api/inference/submit/``, form-encoded exactly
as the reference UI does), polls ``/api/inference/status/<id>/`` and reports request
throughput, output tokens/s, and p50/p99 end-to-end latency (submit -> completed, including
queueing, dispatch, the worker's continuous batching and the HTTP hops). Two modes:

    closed loop   --concurrency C: C clients, each submits its next request when the last
                  one finished (completion seen by a long poll of the status API, or by
                  polling every --poll seconds as the reference UI does every 2 s)
    open loop     --rate R: Poisson arrivals at R requests/s

    python -m distributed_llm_inferencing_amd.loadgen --master http://127.0.0.1:8000 \\
        --model llama3-8b --requests 512 --concurrency 256
"""
from __future__ import annotations

import argparse
import json
import random
import statistics
import threading
import time
from concurrent.futures import ThreadPoolExecutor
from typing import Dict, List, Optional

import requests

WORDS = ("the model runs on eight accelerators and streams tokens back to the dashboard while "
         "the scheduler keeps every pipeline stage busy").split()


def make_prompt(rng: random.Random, words: int) -> str:
    return " ".join(rng.choice(WORDS) for _ in range(words))


class LoadGen:
    def __init__(self, master: str, model: str, session: Optional[requests.Session] = None,
                 poll_s: float = 0.05, timeout_s: float = 600.0):
        self.master = master.rstrip("/")
        self.model = model
        self.http = session or requests.Session()
        if session is None:
            ad = requests.adapters.HTTPAdapter(pool_maxsize=1024)
            self.http.mount("http://", ad)
        self.poll_s, self.timeout_s = poll_s, timeout_s
        self.lock = threading.Lock()
        self.results: List[Dict] = []

    def one(self, prompt: str) -> Dict:
        t0 = time.perf_counter()
        r = self.http.post(f"{self.master}/api/inference/submit/",
                           data={"model_name": self.model, "prompt": prompt}, timeout=30)
        r.raise_for_status()
        rid = r.json()["request_id"]
        st = {}
        while time.perf_counter() - t0 < self.timeout_s:
            if self.poll_s <= 0:          # long poll: the master answers on completion
                st = self.http.get(f"{self.master}/api/inference/status/{rid}/",
                                   params={"wait": 30}, timeout=60).json()
            else:
                st = self.http.get(f"{self.master}/api/inference/status/{rid}/",
                                   timeout=30).json()
            if st.get("status") in ("completed", "failed"):
                break
            if self.poll_s > 0:
                time.sleep(self.poll_s)
        res = {"id": rid, "status": st.get("status", "timeout"),
               "latency_s": time.perf_counter() - t0,
               "execution_time": st.get("execution_time"),
               "result_chars": len(st.get("result") or "")}
        with self.lock:
            self.results.append(res)
        return res

    def closed_loop(self, prompts: List[str], concurrency: int) -> float:
        t0 = time.perf_counter()
        with ThreadPoolExecutor(max_workers=concurrency) as ex:
            list(ex.map(self.one, prompts))
        return time.perf_counter() - t0

    def open_loop(self, prompts: List[str], rate: float, seed: int = 0) -> float:
        rng = random.Random(seed)
        t0 = time.perf_counter()
        threads = []
        for p in prompts:
            th = threading.Thread(target=self.one, args=(p,), daemon=True)
            th.start()
            threads.append(th)
            time.sleep(rng.expovariate(rate))
        for th in threads:
            th.join()
        return time.perf_counter() - t0

    def closed_loop_async(self, prompts: List[str], concurrency: int) -> float:
        """Closed loop on one asyncio loop (aiohttp): C coroutines instead of C threads, so
        the load generator is not the bottleneck of the measurement (the threaded form
        spends ~2 ms of GIL time per request in ``requests``)."""
        import asyncio

        import aiohttp

        async def run() -> float:
            it = iter(prompts)
            conn = aiohttp.TCPConnector(limit=0)
            async with aiohttp.ClientSession(connector=conn) as http:
                async def one(prompt):
                    t0 = time.perf_counter()
                    async with http.post(f"{self.master}/api/inference/submit/",
                                         data={"model_name": self.model, "prompt": prompt},
                                         timeout=aiohttp.ClientTimeout(total=30)) as r:
                        r.raise_for_status()
                        rid = (await r.json())["request_id"]
                    st = {}
                    while time.perf_counter() - t0 < self.timeout_s:
                        params = {"wait": "30"} if self.poll_s <= 0 else None
                        async with http.get(f"{self.master}/api/inference/status/{rid}/",
                                            params=params,
                                            timeout=aiohttp.ClientTimeout(total=60)) as r:
                            st = await r.json()
                        if st.get("status") in ("completed", "failed"):
                            break
                        if self.poll_s > 0:
                            await asyncio.sleep(self.poll_s)
                    self.results.append({"id": rid, "status": st.get("status", "timeout"),
                                         "latency_s": time.perf_counter() - t0,
                                         "execution_time": st.get("execution_time"),
                                         "result_chars": len(st.get("result") or "")})

                async def client():
                    for p in it:
                        await one(p)
                t0 = time.perf_counter()
                await asyncio.gather(*(client() for _ in range(concurrency)))
                return time.perf_counter() - t0
        return asyncio.run(run())

    def report(self, wall_s: float, tokens_per_request: Optional[int] = None) -> Dict:
        ok = [r for r in self.results if r["status"] == "completed"]
        lat = sorted(r["latency_s"] for r in ok)

        def pct(q):
            return lat[min(len(lat) - 1, int(q * len(lat)))] if lat else None
        out = {"requests": len(self.results), "completed": len(ok),
               "failed": len(self.results) - len(ok), "wall_s": round(wall_s, 3),
               "requests_per_s": round(len(ok) / wall_s, 3) if wall_s > 0 else None,
               "p50_latency_s": pct(0.5), "p99_latency_s": pct(0.99),
               "mean_latency_s": statistics.fmean(lat) if lat else None}
        if tokens_per_request:
            out["output_tokens_per_s"] = round(len(ok) * tokens_per_request / wall_s, 2)
        return out


def main(argv=None):
    ap = argparse.ArgumentParser("dli loadgen")
    ap.add_argument("--master", default="http://127.0.0.1:8000")
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--requests", type=int, default=64)
    ap.add_argument("--concurrency", type=int, default=16)
    ap.add_argument("--rate", type=float, default=0.0, help="open loop (requests/s) if > 0")
    ap.add_argument("--prompt-words", type=int, default=24)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--poll", type=float, default=0.0,
                    help="status poll interval (s); 0 = long poll (?wait=30)")
    ap.add_argument("--threads", action="store_true",
                    help="closed loop with one thread per client (default: asyncio)")
    ap.add_argument("--tokens-per-request", type=int, default=0,
                    help="report output tokens/s (requests generate a fixed count)")
    a = ap.parse_args(argv)
    rng = random.Random(a.seed)
    prompts = [make_prompt(rng, a.prompt_words) for _ in range(a.requests)]
    lg = LoadGen(a.master, a.model, poll_s=a.poll)
    if a.rate > 0:
        wall = lg.open_loop(prompts, a.rate, a.seed)
    elif a.threads:
        wall = lg.closed_loop(prompts, a.concurrency)
    else:
        wall = lg.closed_loop_async(prompts, a.concurrency)
    rep = lg.report(wall, a.tokens_per_request or None)
    rep.update(concurrency=a.concurrency, rate=a.rate, poll_s=a.poll)
    print(json.dumps(rep), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
