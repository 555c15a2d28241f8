"""The RCCL (torch.distributed "nccl") branches of fsp_amd.dist, executed for real: a 1-rank
nccl process group on the GPU (one process, no second GPU needed) runs every collective the
trainers use -- init_process_group(device_id=...), all_gather_into_tensor (all_gather_rows,
AllGatherRows forward, GatherClassColumns forward), reduce_scatter_tensor (reduce_scatter_rows,
AllGatherRows backward), the CUDA RNG-state broadcast (sync_rng_from), broadcast_int,
max_over_ranks / sum_over_ranks, allreduce_grads, broadcast_params, all_gather_varlen -- and
the same calls under gloo in the same process; both must give identical results.

Replaces: PromptSRC/trainers/coop.py:435-436 and cocoop.py:308-311 (nn.DataParallel)."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

PROBE = r"""
import json, os, socket, sys
import torch
import torch.distributed as td
sys.path.insert(0, os.environ["FSP_ROOT"])
from fsp_amd import dist

def port():
    s = socket.socket(); s.bind(("127.0.0.1", 0)); p = s.getsockname()[1]; s.close(); return p

def suite():
    dev = torch.device("cuda", 0)
    g = torch.Generator(device="cpu").manual_seed(7)
    x = torch.randn(5, 4, generator=g).to(dev)
    out = {"backend": td.get_backend(), "world": dist.world_size()}
    out["gather_rows"] = dist.all_gather_rows(x, [5]).cpu().tolist()
    out["reduce_scatter"] = dist.reduce_scatter_rows(x * 2, [5]).cpu().tolist()
    a = x.clone().requires_grad_(True)
    y = dist.AllGatherRows.apply(a, [5])
    (y * torch.arange(20, device=dev, dtype=torch.float32).view(5, 4)).sum().backward()
    out["agr_fwd"] = y.detach().cpu().tolist()
    out["agr_bwd"] = a.grad.cpu().tolist()
    b = x.t().contiguous().requires_grad_(True)  # [B=4, C_r=5] logits
    z = dist.GatherClassColumns.apply(b, [5])
    (z * 3).sum().backward()
    out["gcc_fwd"] = z.detach().cpu().tolist()
    out["gcc_bwd"] = b.grad.cpu().tolist()
    torch.manual_seed(1234)
    dist.sync_rng_from(0)
    out["rng_after_sync"] = torch.rand(3).tolist()
    out["bcast_int"] = dist.broadcast_int(41)
    out["max"] = dist.max_over_ranks(2.5)
    out["sum"] = dist.sum_over_ranks(1.5)
    p = torch.nn.Parameter(torch.ones(3, device=dev))
    p.grad = torch.full((3,), 4.0, device=dev)
    dist.allreduce_grads([p])
    out["allreduce"] = p.grad.cpu().tolist()
    dist.broadcast_params([p])
    out["bcast_params"] = p.detach().cpu().tolist()
    out["varlen"] = dist.all_gather_varlen(x[:3]).cpu().tolist()
    import bench  # its N > 1 grad_allreduce field, through this backend
    r = bench.time_grad_allreduce([torch.nn.Parameter(torch.zeros(7, device=dev))], iters=3, warmup=1)
    out["ar_timer"] = [r["bytes"], r["iters"], r["us_per_call"] > 0]
    dist.barrier()
    torch.cuda.synchronize()
    return out

res = {}
os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port()), RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
dist.init_from_env("nccl")  # the production init: device_id bound, backend nccl (RCCL)
res["nccl"] = suite()
td.destroy_process_group()
os.environ["MASTER_PORT"] = str(port())
dist.init_from_env("gloo")
res["gloo"] = suite()
td.destroy_process_group()
print("RESULT " + json.dumps(res))
"""


def test_rccl_branches_one_rank_match_gloo():
    env = dict(os.environ, FSP_ROOT=ROOT, HSA_ENABLE_IPC_MODE_LEGACY="0")
    p = subprocess.run([sys.executable, "-c", PROBE], env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    line = [l for l in p.stdout.splitlines() if l.startswith("RESULT ")][-1]
    res = json.loads(line[len("RESULT "):])
    nc, gl = res["nccl"], res["gloo"]
    assert nc["backend"] == "nccl" and gl["backend"] == "gloo" and nc["world"] == 1
    for k in nc:
        if k in ("backend",):
            continue
        np.testing.assert_array_equal(np.asarray(nc[k]), np.asarray(gl[k]), err_msg=k)
    # 1-rank semantics: gathers are identity, reductions of one rank are the rank's value
    x = np.asarray(nc["gather_rows"])
    np.testing.assert_array_equal(np.asarray(nc["reduce_scatter"]), 2 * x)
    np.testing.assert_array_equal(np.asarray(nc["agr_bwd"]), np.arange(20, dtype=np.float32).reshape(5, 4))
    np.testing.assert_array_equal(np.asarray(nc["gcc_fwd"]), x.T)
    np.testing.assert_array_equal(np.asarray(nc["gcc_bwd"]), np.full((4, 5), 3.0))
    assert nc["bcast_int"] == 41 and nc["max"] == 2.5 and nc["sum"] == 1.5
    assert nc["allreduce"] == [4.0, 4.0, 4.0]
    assert nc["ar_timer"] == [28, 3, True]
