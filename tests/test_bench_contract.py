"""bench.py driver contract on CPU: the driver launches ``python bench.py`` for N = 1 and
``python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N`` for N > 1 and
parses ONE JSON line from rank 0. These runs use a tiny Llama / Mixtral so the same code
paths (single engine, layer-sharded pipeline, DP replicas, expert parallel) finish in
seconds over gloo."""
from __future__ import annotations

import json
import os
import socket
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
        "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config"}


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(cmd, timeout=240):
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="",
               OMP_NUM_THREADS="2")
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True,
                       timeout=timeout)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]      # rank 0 prints exactly one JSON line
    return json.loads(lines[0])


def _check(rec, n, steps, warmup, parallelism):
    assert KEYS <= set(rec)
    assert rec["n_gpus"] == n and rec["steps"] == steps and rec["warmup"] == warmup
    assert rec["value"] > 0 and rec["ms_per_step"] > 0
    assert rec["higher_is_better"] is True and rec["scaling"] == "weak"
    assert rec["dtype"] == "bf16" and rec["unit"] == "tokens/s"
    assert rec["config"]["parallelism"] == parallelism
    assert rec["config"]["seq_len"] == 100
    # whole-job tokens/s: every request generates max_length - prompt_len tokens
    per_wave = rec["config"]["global_batch"] * (100 - rec["config"]["prompt_len"])
    assert rec["value"] == pytest.approx(per_wave * steps / (rec["ms_per_step"] * steps / 1e3),
                                         rel=0.02)


COMMON = ["--batch", "4", "--max-model-len", "128", "--steps", "1", "--warmup", "1"]


def test_bench_single_cpu():
    rec = _run([sys.executable, "bench.py", "--model", "llama-tiny", *COMMON])
    _check(rec, 1, 1, 1, "single")
    assert rec["config"]["global_batch"] == 4


@pytest.mark.parametrize("mode,model,par,gb", [
    ("pp", "llama-tiny", "pp2", 12),        # M = N + 1 microbatches of --batch
    ("dp", "llama-tiny", "dp2", 8),
    ("ep", "mixtral-tiny", "dp2-ep2", 8),   # DP attention + EP experts
])
def test_bench_torchrun_two_ranks(mode, model, par, gb):
    rec = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                "--nproc-per-node", "2", "--master-addr", "127.0.0.1",
                "--master-port", str(_free_port()), "bench.py", "--gpus", "2",
                "--model", model, "--mode", mode, *COMMON])
    _check(rec, 2, 1, 1, par)
    assert rec["config"]["global_batch"] == gb


def test_bench_spawns_its_own_ranks():
    """The driver's plain form ``python bench.py --gpus N`` (no torchrun): bench.py starts
    the N ranks itself and rank 0's line names the data plane and every rank's device."""
    rec = _run([sys.executable, "bench.py", "--gpus", "2", "--model", "llama-tiny",
                "--mode", "pp", *COMMON])
    _check(rec, 2, 1, 1, "pp2")
    assert rec["config"]["global_batch"] == 12
    assert rec["launcher"] == "spawn" and rec["ranks"] == 2
    assert rec["data_plane"] in ("torch-gloo", "ipc-host")
    assert [d["rank"] for d in rec["rank_devices"]] == [0, 1]


def test_spawn_failure_ends_the_job():
    """One rank failing stops the others and the parent returns its exit code (no hang on
    a peer that waits forever for the dead rank)."""
    import time
    from distributed_llm_inferencing_amd import launch
    code = ("import os, sys, time\n"
            "r = int(os.environ['RANK'])\n"
            "assert os.environ['MASTER_ADDR'] == '127.0.0.1' and os.environ['WORLD_SIZE'] == '3'\n"
            "sys.exit(7) if r == 1 else time.sleep(120)\n")
    t0 = time.monotonic()
    rc = launch.spawn([sys.executable, "-c", code], 3)
    assert rc == 7
    assert time.monotonic() - t0 < 60

