"""Debug modes: serialised kernels and per-op fault attribution.

    DLI_DEBUG_SYNC=1   every native op synchronises after launch and reports its own name
                       when a kernel faulted (ops/_native.py); graphs are disabled
    enable_debug_sync() sets that plus AMD_SERIALIZE_KERNEL=3 / AMD_SERIALIZE_COPY=3 and
                       HIP_LAUNCH_BLOCKING=1 — call it before anything initialises HIP.

Host-side sanitizers for the C++ runtime: ``python -m distributed_llm_inferencing_amd.build
--asan-selftest`` (AddressSanitizer on the host code only; GPU ASan / XNACK are not
available on the target pool).
"""
from __future__ import annotations

import os


def enable_debug_sync() -> None:
    os.environ["DLI_DEBUG_SYNC"] = "1"
    os.environ.setdefault("AMD_SERIALIZE_KERNEL", "3")
    os.environ.setdefault("AMD_SERIALIZE_COPY", "3")
    os.environ.setdefault("HIP_LAUNCH_BLOCKING", "1")


def debug_sync_enabled() -> bool:
    return os.environ.get("DLI_DEBUG_SYNC", "0") == "1"
