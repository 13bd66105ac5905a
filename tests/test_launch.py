"""Launchers: serve-node's worker command lines and the data-plane fields a multi-rank
worker reports (per-GPU isolation must not defeat the peer data plane)."""
from __future__ import annotations

import os

from distributed_llm_inferencing_amd import cli, launch


def test_serve_node_keeps_every_gpu_visible(monkeypatch):
    monkeypatch.delenv("HIP_VISIBLE_DEVICES", raising=False)
    monkeypatch.delenv("ROCR_VISIBLE_DEVICES", raising=False)
    monkeypatch.delenv("CUDA_VISIBLE_DEVICES", raising=False)
    cmds = cli.node_commands(4, base_port=6000)
    assert len(cmds) == 4
    for i, (cmd, env) in enumerate(cmds):
        assert "HIP_VISIBLE_DEVICES" not in env and "ROCR_VISIBLE_DEVICES" not in env
        assert "CUDA_VISIBLE_DEVICES" not in env
        assert cmd[cmd.index("--gpu") + 1] == str(i)
        assert cmd[cmd.index("--port") + 1] == str(6000 + i)
        assert env["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
        assert not any("VISIBLE_DEVICES" in c for c in cmd)


def test_serve_node_passes_the_operator_mask_through(monkeypatch):
    """ADVICE r5 (cli.py:46): a preset mask is kept, --gpu i indexes into it, and every GPU
    of the mask stays visible to every worker."""
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "4,5,6,7")
    for i, (cmd, env) in enumerate(cli.node_commands(4)):
        assert env["HIP_VISIBLE_DEVICES"] == "4,5,6,7"
        assert cmd[cmd.index("--gpu") + 1] == str(i)


def test_visible_gpus_never_initialises_hip(monkeypatch, tmp_path):
    """ADVICE r5 (launch.py:134): the parent counts GPUs from the KFD topology under the
    visibility masks; torch's device count (hipGetDeviceCount when amdsmi is missing) is
    never called, and launch.start refuses a parent that already initialised HIP."""
    import torch
    for n, gid in enumerate([0, 1111, 2222, 3333]):          # node 0 = the CPU
        d = tmp_path / str(n)
        d.mkdir()
        (d / "gpu_id").write_text(f"{gid}\n")
    calls = []
    monkeypatch.setattr(torch.cuda, "device_count", lambda: calls.append(1) or 8)
    monkeypatch.setattr(torch._C, "_cuda_getDeviceCount", lambda: calls.append(2) or 8,
                        raising=False)
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(var, raising=False)
    assert launch.kfd_gpus(str(tmp_path)) == 3
    monkeypatch.setattr(launch, "kfd_gpus", lambda: 3)
    assert launch.visible_gpus() == 3
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "2,0")
    assert launch.visible_gpus() == 2
    monkeypatch.setenv("ROCR_VISIBLE_DEVICES", "1")
    assert launch.visible_gpus() == 0          # HIP's "2,0" names a device ROCR hid
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "0")
    assert launch.visible_gpus() == 1
    assert calls == []
    monkeypatch.setattr(torch.cuda, "is_initialized", lambda: True)
    import pytest
    with pytest.raises(RuntimeError, match="initialised the GPU"):
        launch.start(["true"], 1)


def test_rank_env_is_torchrun_compatible():
    env = launch.rank_env({"X": "1"}, 2, 4, 29999)
    assert env["RANK"] == "2" and env["LOCAL_RANK"] == "2" and env["WORLD_SIZE"] == "4"
    assert env["MASTER_ADDR"] == "127.0.0.1" and env["MASTER_PORT"] == "29999"
    assert env["X"] == "1" and env["DLI_LAUNCHER"] == "spawn"


def test_under_launcher(monkeypatch):
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.delenv("RANK", raising=False)
    assert not launch.under_launcher()
    monkeypatch.setenv("WORLD_SIZE", "2")
    monkeypatch.setenv("RANK", "0")
    assert launch.under_launcher()


def test_data_plane_names():
    from distributed_llm_inferencing_amd.parallel.transport import (data_plane_name,
                                                                    distinct_gpus)
    assert data_plane_name("ipc", True) == "ipc"
    assert data_plane_name("ipc", False) == "ipc-host"
    assert data_plane_name("rccl", True) == "rccl"
    assert data_plane_name("torch", True) == "torch-rccl"
    assert data_plane_name("torch", False) == "torch-gloo"
    same = [{"host": "h", "device": "cuda:0", "pci": "0000:05:00"}] * 2
    assert distinct_gpus(same) == 1
    two = [{"host": "h", "device": "cuda:0", "pci": "0000:05:00"},
           {"host": "h", "device": "cuda:1", "pci": "0000:15:00"}]
    assert distinct_gpus(two) == 2
    assert distinct_gpus([{"host": "h", "device": "cpu"}]) == 0
