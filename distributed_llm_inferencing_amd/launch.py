"""Single-node rank launcher: N child processes, one per GPU, with the torchrun environment
(RANK / LOCAL_RANK / WORLD_SIZE / LOCAL_WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT).

The reference's "nodes" are separately started worker processes behind the master
(``/root/reference/docker-compose.yml:27-55``); here one 8-GPU host runs one process per
MI355X. ``bench.py --gpus N`` and ``cli serve-expert`` call :func:`spawn` when they are not
already running under torchrun, so the plain command form launches every rank itself.

Rules this module keeps (they matter on a GPU box):

* the parent never touches the GPU (no HIP call before or after the fork: the children are
  fresh interpreters started with fork+exec of ``sys.executable``);
* the children share the parent's process group, so a ``timeout`` around the parent reaches
  them too, and each child gets ``PR_SET_PDEATHSIG`` = SIGKILL so none outlives a parent that
  was killed outright;
* the first child that exits non-zero ends the run: the others are terminated (exact PIDs,
  SIGTERM then SIGKILL after a grace period) and the parent returns that child's code.
"""
from __future__ import annotations

import ctypes
import os
import signal
import socket
import subprocess
import sys
import time
from typing import Dict, List, Optional, Sequence

_PR_SET_PDEATHSIG = 1


def under_launcher() -> bool:
    """True when this process already is one rank of a launched job (torchrun or spawn)."""
    return "WORLD_SIZE" in os.environ and "RANK" in os.environ


def free_port(host: str = "127.0.0.1") -> int:
    """A TCP port nothing listens on right now (the rendezvous store binds it next)."""
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind((host, 0))
        return int(s.getsockname()[1])


def rank_env(base: Dict[str, str], rank: int, world: int, port: int,
             local_rank: Optional[int] = None) -> Dict[str, str]:
    env = dict(base)
    lr = rank if local_rank is None else local_rank
    env.update(RANK=str(rank), LOCAL_RANK=str(lr), WORLD_SIZE=str(world),
               LOCAL_WORLD_SIZE=str(world), GROUP_RANK="0", MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(port), DLI_LAUNCHER="spawn")
    # the host driver supports dmabuf IPC only (RCCL + the IPC mailboxes need it)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return env


def _pdeathsig() -> None:                       # runs in the child between fork and exec
    try:
        ctypes.CDLL("libc.so.6", use_errno=True).prctl(_PR_SET_PDEATHSIG, signal.SIGKILL)
    except Exception:  # noqa: BLE001 — best effort; the process group still reaches us
        pass


def start(cmd: Sequence[str], world: int, env: Optional[Dict[str, str]] = None,
          port: Optional[int] = None) -> List[subprocess.Popen]:
    """Start ``world`` copies of ``cmd``, rank r with the torchrun variables of rank r."""
    tm = sys.modules.get("torch")
    if tm is not None and tm.cuda.is_initialized():
        raise RuntimeError("launch.start: this process has initialised the GPU; its ranks "
                           "must be started before any HIP call (fork after HIP init)")
    port = port or free_port()
    base = dict(os.environ if env is None else env)
    procs = []
    for r in range(world):
        procs.append(subprocess.Popen(list(cmd), env=rank_env(base, r, world, port),
                                      preexec_fn=_pdeathsig))
    return procs


def stop(procs: Sequence[subprocess.Popen], grace_s: float = 10.0) -> None:
    """Terminate every still-running child (exact PIDs), then kill what ignores SIGTERM."""
    for p in procs:
        if p.poll() is None:
            try:
                p.terminate()
            except ProcessLookupError:
                pass
    t0 = time.monotonic()
    for p in procs:
        left = max(0.0, grace_s - (time.monotonic() - t0))
        try:
            p.wait(timeout=left)
        except subprocess.TimeoutExpired:
            p.kill()
            p.wait()


def wait(procs: Sequence[subprocess.Popen], poll_s: float = 0.2) -> int:
    """Wait for every child. The first non-zero exit ends the job (the rest are stopped)
    and is returned; 0 when all succeed. SIGTERM / SIGINT to the parent stop the children."""
    stopping = {"sig": None}

    def _on_signal(sig, _frame):
        stopping["sig"] = sig

    old = {s: signal.signal(s, _on_signal) for s in (signal.SIGTERM, signal.SIGINT)}
    try:
        while True:
            if stopping["sig"] is not None:
                stop(procs)
                return 128 + int(stopping["sig"])
            codes = [p.poll() for p in procs]
            bad = [c for c in codes if c not in (None, 0)]
            if bad:
                stop(procs)
                return bad[0] if bad[0] > 0 else 128 - bad[0]
            if all(c == 0 for c in codes):
                return 0
            time.sleep(poll_s)
    finally:
        for s, h in old.items():
            signal.signal(s, h)


def spawn(cmd: Sequence[str], world: int, env: Optional[Dict[str, str]] = None,
          port: Optional[int] = None) -> int:
    """Run ``world`` ranks of ``cmd`` to completion; returns the job's exit code."""
    return wait(start(cmd, world, env=env, port=port))


def spawn_self(world: int, argv: Optional[Sequence[str]] = None,
               env: Optional[Dict[str, str]] = None) -> int:
    """Re-run this script (``sys.argv[0]`` with ``argv``) as ``world`` ranks."""
    args = list(sys.argv[1:] if argv is None else argv)
    return spawn([sys.executable, "-u", os.path.abspath(sys.argv[0]), *args], world, env=env)


def _visibility_mask(n: int) -> int:
    """Apply ROCR_VISIBLE_DEVICES, then HIP_VISIBLE_DEVICES / CUDA_VISIBLE_DEVICES (the HIP
    runtime's order) to ``n`` devices: how many of them a child would see."""
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is None:
            continue
        ids = [t.strip() for t in v.split(",") if t.strip()]
        keep = 0
        for t in ids:
            if t.lstrip("-").isdigit():
                i = int(t)
                if i < 0 or i >= n:      # the runtime stops at the first invalid entry
                    break
            keep += 1                    # UUID-style entries: trust them
        n = min(n, keep)
    return n


def kfd_gpus(topology: str = "/sys/class/kfd/kfd/topology/nodes") -> int:
    """GPU agents in the KFD topology (nodes whose ``gpu_id`` is non-zero; CPU nodes have
    0): a sysfs read, no HIP / HSA call."""
    n = 0
    try:
        for node in sorted(os.listdir(topology)):
            try:
                with open(os.path.join(topology, node, "gpu_id")) as f:
                    if int(f.read().strip() or "0") != 0:
                        n += 1
            except (OSError, ValueError):
                continue
    except OSError:
        return 0
    return n


def visible_gpus() -> int:
    """GPUs this process could hand to its children, counted WITHOUT initialising HIP: the
    KFD topology in sysfs under the HIP / ROCR visibility masks. (``torch.cuda.device_count``
    reads amdsmi on this image, but falls back to ``hipGetDeviceCount`` — a HIP init in the
    parent that then forks its ranks — when amdsmi is unavailable, so it is never used.)"""
    return _visibility_mask(kfd_gpus())
