"""bench.py's driver contract on the CPU: --gpus N starts N ranks itself (torchrun as a child
process, before anything touches the GPU), and a process group that does not match --gpus is
refused; the metric label follows --arch."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_launcher_command_line():
    cmd = bench.launcher_cmd(["--gpus", "8", "--steps", "5"], 8, 29511)
    assert cmd[0] == sys.executable and cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nnodes=1" in cmd and "--nproc-per-node=8" in cmd and "--master-port=29511" in cmd
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1"
    assert cmd[-5] == os.path.join(ROOT, "bench.py")
    assert cmd[-4:] == ["--gpus", "8", "--steps", "5"]


def test_gpus_n_spawns_ranks_as_a_child(monkeypatch):
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    calls = []
    monkeypatch.setattr(subprocess, "call", lambda cmd, env=None: calls.append((cmd, env)) or 3)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4", "--steps", "2"])
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert e.value.code == 3  # the child's return code is relayed
    cmd, env = calls[0]
    assert "--nproc-per-node=4" in cmd and cmd[-4:] == ["--gpus", "4", "--steps", "2"]
    assert env["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"


def test_world_must_match_gpus(monkeypatch):
    monkeypatch.setenv("WORLD_SIZE", "1")  # a torchrun env of one rank
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "2"])
    with pytest.raises(SystemExit, match="--gpus 2 but the process group has 1 ranks"):
        bench.main()


def test_metric_label_follows_arch():
    assert bench.metric_name("ViT-B/16") == \
        "CoCoOp ViT-B/16 16-shot train-step images/sec at 1/2/4/8 GPUs; eval images/sec"
    assert "ViT-L/14@336px" in bench.metric_name("ViT-L/14@336px")
