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


def test_kernel_table_bound_from_intensity():
    """Each kernel class's roofline bound comes from its own FLOP/byte ratio against the ridge
    point (peak / 8 TB/s), not a fixed label: a K = 512 GEMM whose bytes outweigh its FLOPs is
    HBM-bound, a K = 2,048 one MFMA-bound, attention / LayerNorm (no FLOPs counted) HBM-bound."""
    sites = {  # site: (total ms, launches, flops, bytes)
        "text.out_fwd": (0.5, 12, 12 * 24.7e9, 12 * 150e6),     # 165 FLOP/B < 312
        "text.fc_dx": (1.0, 12, 12 * 98.9e9, 12 * 200e6),       # 495 FLOP/B > 312
        "text.attn_bwd": (1.0, 12, 0.0, 12 * 350e6),
    }
    t = bench.kernel_table(sites, 1, "fp16")
    assert t["gemm_out_fwd"]["bound"] == "hbm"
    assert abs(t["gemm_out_fwd"]["roof_frac"] - t["gemm_out_fwd"]["hbm_frac"]) < 1e-9
    assert t["gemm_dx_n512"]["bound"] == "mfma"
    assert abs(t["gemm_dx_n512"]["roof_frac"] - t["gemm_dx_n512"]["mfma_frac"]) < 1e-9
    assert t["attn_bwd"]["bound"] == "hbm"
    r = bench.roofline_of(t, "fp16")
    assert r["kernel_class"] == "gemm_dx_n512" and r["bound"] == "mfma"
