"""Launchers: serve-node's worker command lines and the data-plane fields a multi-rank
worker reports (per-GPU isolation must not defeat the peer data plane)."""
from __future__ import annotations

import os

from distributed_llm_inferencing_amd import cli, launch


def test_serve_node_keeps_every_gpu_visible(monkeypatch):
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "3")
    cmds = cli.node_commands(4, base_port=6000)
    assert len(cmds) == 4
    for i, (cmd, env) in enumerate(cmds):
        assert "HIP_VISIBLE_DEVICES" not in env and "ROCR_VISIBLE_DEVICES" not in env
        assert "CUDA_VISIBLE_DEVICES" not in env
        assert cmd[cmd.index("--gpu") + 1] == str(i)
        assert cmd[cmd.index("--port") + 1] == str(6000 + i)
        assert env["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
        assert not any("VISIBLE_DEVICES" in c for c in cmd)


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
