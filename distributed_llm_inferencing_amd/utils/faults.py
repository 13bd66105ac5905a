"""Fault injection (the reference had none).

``DLI_FAULT`` holds comma-separated rules ``site:action[:arg]``; every component calls
``check(site, **ctx)`` at its injection point:

    worker.inference:error[:p]       raise (HTTP 500) with probability p (default 1)
    worker.inference:delay:<ms>      sleep before serving
    worker.inference:exit_after:<n>  hard-exit the worker process after n requests (node death)
    worker.health:error[:p]          /health answers 503 (drives the failure detector)
    transport.exchange:error:<tick>  the pipeline transport raises at that tick (link failure)
    pipeline.stage:exit_after:<n>    a non-head pipeline rank hard-exits after n ticks (GPU /
                                     process death mid-session)
    dispatch.post:error[:p]          the master's HTTP call to a worker fails (connection error)

Rules are parsed once per process (``reload()`` re-reads the variable, used by tests).
"""
from __future__ import annotations

import os
import random
import threading
import time
from dataclasses import dataclass
from typing import Dict, List


class InjectedFault(RuntimeError):
    pass


@dataclass
class Rule:
    site: str
    action: str
    arg: str = ""
    hits: int = 0


_rules: List[Rule] = []
_lock = threading.Lock()
_loaded = False


def reload(spec: str = None) -> None:
    global _rules, _loaded
    spec = os.environ.get("DLI_FAULT", "") if spec is None else spec
    rules = []
    for part in [p.strip() for p in spec.split(",") if p.strip()]:
        bits = part.split(":")
        if len(bits) < 2:
            continue
        rules.append(Rule(bits[0], bits[1], ":".join(bits[2:])))
    with _lock:
        _rules = rules
        _loaded = True


def active() -> bool:
    if not _loaded:
        reload()
    return bool(_rules)


def check(site: str, **ctx) -> None:
    if not _loaded:
        reload()
    if not _rules:
        return
    for r in _rules:
        if r.site != site:
            continue
        with _lock:
            r.hits += 1
            hits = r.hits
        if r.action == "error":
            if site == "transport.exchange":
                if r.arg and int(ctx.get("tick", -1)) != int(r.arg):
                    continue
                raise InjectedFault(f"injected fault at {site} tick {ctx.get('tick')}")
            p = float(r.arg) if r.arg else 1.0
            if random.random() < p:
                raise InjectedFault(f"injected fault at {site}")
        elif r.action == "delay":
            time.sleep(float(r.arg or 0) / 1000.0)
        elif r.action == "exit_after":
            if hits > int(r.arg or 0):
                os._exit(17)


def stats() -> Dict[str, int]:
    return {f"{r.site}:{r.action}": r.hits for r in _rules}
