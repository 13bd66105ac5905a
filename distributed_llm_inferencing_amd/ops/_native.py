"""ctypes bindings for ``lib/libdli_kernels.so`` (the gfx950 HIP kernels).

The library exposes a plain C ABI (``extern "C" int dli_*(..., hipStream_t)``); every call
passes raw device pointers and torch's *current* HIP stream, so the kernels order correctly
with torch's own work and are captured by ``torch.cuda.CUDAGraph`` (= hipGraph on ROCm).

Loading policy: ``import torch`` first so torch's ``libamdhip64.so.7`` is the one our
library binds to (same SONAME, one HIP runtime per process). On a GPU host a missing or
stale library is an error, never a silent fallback (see ``require_native``).
"""
from __future__ import annotations

import ctypes
import os
import threading
from pathlib import Path

import torch

LIB_PATH = Path(__file__).resolve().parent.parent / "lib" / "libdli_kernels.so"

_lock = threading.Lock()
_lib = None
_load_error: Exception | None = None

P = ctypes.c_void_p
I = ctypes.c_int
F = ctypes.c_float
L = ctypes.c_long

_SIGS = {
    "dli_rmsnorm": [P, P, P, P, I, I, F, P],
    "dli_fused_add_rmsnorm": [P, P, P, P, I, I, F, P],
    "dli_layernorm": [P, P, P, P, P, I, I, F, P],
    "dli_fused_add_layernorm": [P, P, P, P, P, I, I, F, P],
    "dli_rope_cache": [P, I, P, P, P, P, P, I, I, I, I, I, I, P],
    "dli_embedding": [P, P, P, P, P, I, I, P],
    "dli_silu_mul": [P, P, I, I, P],
    "dli_bias_act": [P, P, I, I, I, P],
    "dli_feed_ids": [P, P, P, I, I, P],
    "dli_prefetch": [P, L, I, P, P],
    "dli_decode_attention": [P, P, I, P, P, P, I, P, I, I, I, I, I, F, I, I, P, P],
    "dli_decode_attention_workspace_bytes": [I, I, I, I],
    "dli_prefill_attention": [P, I, P, I, P, I, I, I, I, I, F, P],
    "dli_prefill_set_min_len": [I],
    "dli_prefill_set_pack": [I],
    "dli_sample_set_split_max_b": [I],
    "dli_decode_set_pipe": [I],
    "dli_decode_get_pipe": [],
    "dli_decode_set_form": [I],
    "dli_gemm_set_slab_store": [I],
    "dli_gemm_set_slab_store_family": [I, I],
    "dli_prefill_attention_paged": [P, I, P, I, P, P, P, P, P, I, I, I, I, I, I, I, F, P],
    "dli_sample": [P, P, L, I, I, P, P, P, P, P, P],
    "dli_sample_workspace_bytes": [I, I],
    "dli_sample_bf16": [P, P, L, I, I, P, P, P, P, P, P],
    "dli_topk_rows_bf16": [P, P, P, L, I, I, I, I, P],
    "dli_topk_rows": [P, P, P, L, I, I, I, I, P],
    "dli_gemm": [P, I, P, I, P, I, I, I, I, I, I, I, P, P, P, I, P],
    "dli_splitk_add_rmsnorm": [P, P, P, I, I, I, P, F, I, P],
    "dli_gemv_fused": [P, I, P, F, P, I, P, I, I, I, I, I, I, I, P, P],
    "dli_splitk_rope_cache": [P, P, I, I, I, P, P, P, P, P, I, I, I, I, I, I, P],
    "dli_decode_attention_fused": [P, P, I, P, P, P, P, P, P, I, P, I, I, I, I, I, F, I, P],
    "dli_moe_route": [P, P, P, I, I, I, P],
    "dli_moe_router": [P, P, P, I, P, I, I, I, I, P],
    "dli_splitk_add_rmsnorm_route": [P, P, P, I, I, I, P, F, P, I, I, P, P, P],
    "dli_moe_align": [P, P, P, P, I, I, I, I, P],
    "dli_moe_gather": [P, P, P, I, I, P, P],
    "dli_moe_combine": [P, P, P, P, I, I, I, P],
    "dli_moe_combine_slabs": [P, P, I, I, P, P, I, I, I, P],
    "dli_moe_combine_add_rmsnorm": [P, P, P, I, I, P, P, I, I, I, P, F, P],
    "dli_gemm_grouped_gather": [P, I, P, I, P, I, I, I, I, I, P, P, I, P],
    "dli_ep_pack": [P, P, P, P, P, P, P, I, I, I, I, P],
}


def ensure_current(lib_path: Path, kind: str) -> None:
    """Build a missing library, rebuild a stale one (its source-digest stamp does not match
    the tree), and refuse a stale one when no toolchain can rebuild it."""
    from .. import build as _build
    if _build.is_current(kind, lib_path):
        return
    try:
        _build._hipcc()
    except RuntimeError:
        if lib_path.exists():
            raise RuntimeError(f"{lib_path} is stale (sources changed since it was built; "
                               f"stamp {_build.stamp_path(lib_path).name}) and hipcc is not "
                               "available to rebuild it")
        raise
    _build.build(verbose=False)
    if not _build.is_current(kind, lib_path):
        raise RuntimeError(f"{lib_path} still does not match its sources after a rebuild")


def _load():
    global _lib, _load_error
    with _lock:
        if _lib is not None or _load_error is not None:
            return _lib
        try:
            ensure_current(LIB_PATH, "kernels")
            lib = ctypes.CDLL(str(LIB_PATH))
            for name, args in _SIGS.items():
                fn = getattr(lib, name)
                fn.argtypes = args
                fn.restype = ctypes.c_long if name.endswith("_bytes") else ctypes.c_int
            _lib = lib
        except Exception as e:  # noqa: BLE001 - surfaced by require_native()
            _load_error = e
        return _lib


def available() -> bool:
    return _load() is not None


def load_error() -> Exception | None:
    _load()
    return _load_error


def require_native():
    lib = _load()
    if lib is None:
        raise RuntimeError(
            f"HIP kernel library {LIB_PATH} could not be loaded ({_load_error}); "
            "run `python -m distributed_llm_inferencing_amd.build` — refusing to fall back "
            "to PyTorch ops on a GPU")
    return lib


def stream_ptr() -> int:
    return torch.cuda.current_stream().cuda_stream


def ptr(t) -> int | None:
    return None if t is None else t.data_ptr()


# DLI_DEBUG_SYNC=1: synchronise after every native launch and name the op whose kernel
# faulted (SURVEY.md §5.2 debug mode; pair with AMD_SERIALIZE_KERNEL=3 set before HIP init,
# which utils.debug.enable_debug_sync() does). Not usable inside hipGraph capture.
_DEBUG_SYNC = os.environ.get("DLI_DEBUG_SYNC", "0") == "1"


def call(name: str, *args) -> None:
    lib = require_native()
    rc = getattr(lib, name)(*args)
    if rc != 0:
        raise RuntimeError(f"{name} failed with hipError {rc}")
    if _DEBUG_SYNC:
        import torch
        if not torch.cuda.is_current_stream_capturing():
            try:
                torch.cuda.synchronize()
            except RuntimeError as e:
                raise RuntimeError(f"{name}: kernel fault detected after launch: {e}") from e


def loaded_path() -> str | None:
    return str(LIB_PATH) if _lib is not None else None


