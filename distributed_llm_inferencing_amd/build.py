"""In-tree native build: hipcc for gfx950, no torch headers, no JIT cache.

Produces two shared objects inside the package (they travel to the GPU box with the
repo snapshot; they are git-ignored):

* ``lib/libdli_kernels.so`` — every HIP/CDNA4 kernel in ``csrc/kernels`` behind a plain
  ``extern "C"`` ABI (called through ctypes with torch's current HIP stream).
* ``lib/libdli_runtime.so`` — the host-side C++ runtime in ``csrc/runtime``: paged-KV block
  allocator + batched block-table / slot builders (``block_manager.cpp``), the decode fast
  path of the continuous-batching scheduler (``decode_core.cpp``), the safetensors weight
  loader with pinned staging + hipMemcpyAsync (``safetensors_loader.cpp``), the
  pipeline's shared-memory control ring (``shm_ring.cpp``) and its optional RCCL data
  plane (``comm.cpp``: grouped ncclSend/ncclRecv on the compute stream, ``DLI_PP_COMM=rccl``).

Each library is stamped with a digest of its sources + flags (``<lib>.sha1``); the loaders
(``ops/_native.py``, ``runtime/__init__.py``) rebuild a library whose stamp does not match
the tree, or refuse to load it when no toolchain is present — never a stale binary.

Both link ``libamdhip64.so.7``; at run time the copy torch already loaded is reused
(same SONAME), so kernels launched here and torch's own kernels share one HIP runtime.

Usage: ``python -m distributed_llm_inferencing_amd.build [--force] [-j N]``
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import hashlib
import os
import shutil
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent
REPO = PKG.parent
CSRC = REPO / "csrc"
LIBDIR = PKG / "lib"
OBJDIR = REPO / "build" / "obj"
ARCH = os.environ.get("DLI_OFFLOAD_ARCH", "gfx950")


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and Path(cand).exists():
            return cand
    raise RuntimeError("hipcc not found (set HIPCC or install ROCm)")


# NOTE: no -ffast-math: it implies no-infs, and the attention/sampling kernels rely on
# -inf as the masked-score / running-max sentinel (poison under ninf -> NaNs).
KERNEL_FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-fno-gpu-rdc",
                "-munsafe-fp-atomics", "-Wno-unused-result"]
RUNTIME_FLAGS = ["-O2", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wall",
                 "-Wno-unused-result"]


def _digest(paths, flags) -> str:
    h = hashlib.sha1()
    for p in sorted(paths):
        h.update(p.name.encode())
        h.update(p.read_bytes())
    h.update(" ".join(flags).encode())
    return h.hexdigest()


# Kernels whose MFMAs are inline asm: hipcc pads no hazard after an asm statement, so any
# compiler-made copy of their accumulators inside the K loop (a scratch spill, a rolled
# epilogue indexing them dynamically) reads AGPRs an MFMA may still be writing. Such a
# kernel must keep its accumulators in registers: a nonzero scratch size fails the build.
ASM_MFMA_KERNELS = ("gemm4w_kernel", "gemm4wp_kernel")
_REMARKS = "-Rpass-analysis=kernel-resource-usage"


def check_scratch(stderr: str, src: str) -> None:
    """Raise if a kernel named in ASM_MFMA_KERNELS reports scratch (hipcc resource remarks)."""
    fn = None
    for line in stderr.splitlines():
        if "remark:" not in line:
            continue
        body = line.split("remark:", 1)[1].strip()
        if body.startswith("Function Name:"):
            fn = body.split(":", 1)[1].strip()
        elif body.startswith("ScratchSize") and fn and any(k in fn for k in ASM_MFMA_KERNELS):
            size = int(body.split(":")[-1].split()[0])
            if size:
                raise RuntimeError(f"{src}: {fn} uses {size} B/lane of scratch: its inline-asm "
                                   "MFMA accumulators would be copied without hazard padding")


def _compile(src: Path, obj: Path, flags, headers) -> Path:
    stamp = obj.with_suffix(".sha1")
    dig = _digest([src, *headers], flags)
    if obj.exists() and stamp.exists() and stamp.read_text() == dig:
        return obj
    obj.parent.mkdir(parents=True, exist_ok=True)
    remarks = src.suffix == ".hip" and any(k.split("_")[0] in src.read_text()
                                           for k in ASM_MFMA_KERNELS)
    cmd = [_hipcc(), *flags, *([_REMARKS] if remarks else []), "-I", str(CSRC / "kernels"),
           "-I", str(CSRC / "runtime"), "-c", str(src), "-o", str(obj)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src.name}:\n{' '.join(cmd)}\n{r.stderr[-6000:]}")
    if remarks:
        check_scratch(r.stderr, src.name)
    stamp.write_text(dig)
    return obj


def _link(objs, out: Path, extra=()):
    out.parent.mkdir(parents=True, exist_ok=True)
    tmp = out.with_suffix(".so.tmp")
    cmd = [_hipcc(), "-shared", "-fPIC", f"--offload-arch={ARCH}", *map(str, objs), "-o", str(tmp),
           *extra]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed for {out.name}:\n{r.stderr[-4000:]}")
    os.replace(tmp, out)


def _group_sources(kind: str):
    if kind == "kernels":
        return (sorted((CSRC / "kernels").glob("*.hip")), sorted((CSRC / "kernels").glob("*.h")),
                KERNEL_FLAGS)
    return (sorted((CSRC / "runtime").glob("*.cpp")), sorted((CSRC / "runtime").glob("*.h")),
            RUNTIME_FLAGS)


def source_digest(kind: str) -> str:
    """Digest of one library's sources + headers + flags (``kernels`` or ``runtime``)."""
    srcs, hdrs, flags = _group_sources(kind)
    return _digest([*srcs, *hdrs], flags)


def stamp_path(lib: Path) -> Path:
    return lib.with_name(lib.name + ".sha1")


def is_current(kind: str, lib: Path) -> bool:
    st = stamp_path(lib)
    return lib.exists() and st.exists() and st.read_text().strip() == source_digest(kind)


def _build_group(srcs, headers, flags, out: Path, jobs: int, extra=(), kind=None):
    objs_dir = OBJDIR / out.stem
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        futs = [ex.submit(_compile, s, objs_dir / (s.stem + ".o"), flags, headers) for s in srcs]
        objs = [f.result() for f in futs]
    newest = max(o.stat().st_mtime for o in objs)
    if kind is not None and not is_current(kind, out) or not out.exists() \
            or out.stat().st_mtime < newest:
        _link(objs, out, extra)
    if kind is not None:
        stamp_path(out).write_text(source_digest(kind))
    return out


def build(force: bool = False, jobs: int = 0, verbose: bool = True) -> dict:
    jobs = jobs or min(8, os.cpu_count() or 4)
    if force and OBJDIR.exists():
        shutil.rmtree(OBJDIR)
    k_srcs, k_hdrs, k_flags = _group_sources("kernels")
    r_srcs, r_hdrs, _ = _group_sources("runtime")
    out = {}
    # --no-undefined: a kernel whose host-side handle hipcc failed to emit (it happens
    # silently, e.g. for a lambda capturing an __amdgpu_buffer_rsrc_t) fails the link here
    # instead of the library failing to load on the GPU box
    out["kernels"] = _build_group(k_srcs, k_hdrs, k_flags, LIBDIR / "libdli_kernels.so", jobs,
                                  extra=("-Wl,--no-undefined",), kind="kernels")
    if r_srcs:
        out["runtime"] = _build_group(r_srcs, r_hdrs, RUNTIME_FLAGS, LIBDIR / "libdli_runtime.so",
                                      jobs, extra=("-lpthread",), kind="runtime")
    if verbose:
        for k, v in out.items():
            print(f"[dli.build] {k}: {v} ({v.stat().st_size // 1024} KiB)")
    return out


def build_asan_selftest(verbose: bool = True) -> Path:
    """Host-AddressSanitizer build of the C++ runtime + its self-test driver
    (csrc/runtime/tests/runtime_selftest.cpp). Sanitizer flags are host-only
    (``-Xarch_host``): GPU ASan is not available on the target pool."""
    srcs = sorted((CSRC / "runtime").glob("*.cpp")) + [CSRC / "runtime" / "tests" /
                                                        "runtime_selftest.cpp"]
    out = REPO / "build" / "runtime_selftest_asan"
    out.parent.mkdir(parents=True, exist_ok=True)
    newest = max(p.stat().st_mtime for p in srcs)
    if not out.exists() or out.stat().st_mtime < newest:
        cmd = [_hipcc(), "-O1", "-g", "-std=c++17", "-Xarch_host", "-fsanitize=address",
               "-Xarch_host", "-fno-omit-frame-pointer", *map(str, srcs), "-o", str(out),
               "-lpthread"]
        if verbose:
            print("[dli.build]", " ".join(cmd))
        subprocess.run(cmd, check=True)
    return out


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", type=int, default=0)
    ap.add_argument("--asan-selftest", action="store_true",
                    help="build + run the host-ASan runtime self-test")
    a = ap.parse_args(argv)
    if a.asan_selftest:
        exe = build_asan_selftest()
        env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1")
        return subprocess.run([str(exe)], env=env).returncode
    build(force=a.force, jobs=a.j)


if __name__ == "__main__":
    sys.exit(main())
