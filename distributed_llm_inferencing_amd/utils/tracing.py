"""Tracing / profiling hooks (the reference had only ``execution_time``).

* ``trace_range(name)`` — a roctx range (``roctxRangePushA/Pop`` from the ROCm roctx library)
  when ``DLI_TRACE=1``; rocprofv3 ``--marker-trace`` then shows engine steps, prefill/decode,
  pipeline exchanges and MoE all-to-alls on the timeline next to the kernels. No-op otherwise.
* ``SpanLog`` — per-request spans (queue wait, time to first token, decode time, total, token
  counts) appended as JSON lines to ``logs/requests.jsonl`` when ``DLI_TRACE=1`` or
  ``DLI_REQUEST_LOG`` names a file.
* ``StepTimer`` — cumulative host-side timings of the engine loop phases.
"""
from __future__ import annotations

import contextlib
import ctypes
import json
import os
import threading
import time
from pathlib import Path
from typing import Optional

_ROCTX = None
_ROCTX_TRIED = False


def enabled() -> bool:
    return os.environ.get("DLI_TRACE", "0") == "1"


def _roctx():
    global _ROCTX, _ROCTX_TRIED
    if _ROCTX_TRIED:
        return _ROCTX
    _ROCTX_TRIED = True
    for name in ("librocprofiler-sdk-roctx.so.1", "libroctx64.so.4", "libroctx64.so",
                 "/opt/rocm/lib/librocprofiler-sdk-roctx.so", "/opt/rocm/lib/libroctx64.so"):
        try:
            lib = ctypes.CDLL(name)
            lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
            lib.roctxRangePushA.restype = ctypes.c_int
            lib.roctxRangePop.restype = ctypes.c_int
            lib.roctxMarkA.argtypes = [ctypes.c_char_p]
            _ROCTX = lib
            break
        except (OSError, AttributeError):
            continue
    return _ROCTX


_NULL_RANGE = contextlib.nullcontext()


def trace_range(name: str):
    """roctx range around a block; a shared no-op context when tracing is off (this wraps
    per-tick pipeline operations: no generator per call on the hot path)."""
    if not enabled():
        return _NULL_RANGE
    return _roctx_range(name)


@contextlib.contextmanager
def _roctx_range(name: str):
    lib = _roctx()
    if lib is not None:
        lib.roctxRangePushA(name.encode())
    try:
        yield
    finally:
        if lib is not None:
            lib.roctxRangePop()


def mark(name: str) -> None:
    if enabled():
        lib = _roctx()
        if lib is not None:
            lib.roctxMarkA(name.encode())


class SpanLog:
    _lock = threading.Lock()

    def __init__(self, path: Optional[str] = None):
        if path is None:
            path = os.environ.get("DLI_REQUEST_LOG") or (
                str(Path(os.environ.get("DLI_LOG_DIR", "logs")) / "requests.jsonl")
                if enabled() else None)
        self.path = path
        if path:
            Path(path).parent.mkdir(parents=True, exist_ok=True)

    def record(self, out, **extra) -> None:
        if not self.path:
            return
        rec = {"ts": time.time(), "request_id": out.request_id,
               "prompt_tokens": len(out.prompt_ids), "output_tokens": len(out.output_ids),
               "latency_s": round(out.latency_s, 6),
               "ttft_s": round(out.ttft_s, 6) if out.ttft_s is not None else None,
               "finish_reason": out.finish_reason, **extra}
        with self._lock, open(self.path, "a") as f:
            f.write(json.dumps(rec) + "\n")


class StepTimer:
    def __init__(self):
        self.t = {}
        self.n = {}

    @contextlib.contextmanager
    def phase(self, name: str):
        t0 = time.perf_counter()
        try:
            yield
        finally:
            self.t[name] = self.t.get(name, 0.0) + time.perf_counter() - t0
            self.n[name] = self.n.get(name, 0) + 1

    def snapshot(self) -> dict:
        return {k: {"total_s": round(v, 6), "calls": self.n[k],
                    "avg_us": round(1e6 * v / max(1, self.n[k]), 2)} for k, v in self.t.items()}
