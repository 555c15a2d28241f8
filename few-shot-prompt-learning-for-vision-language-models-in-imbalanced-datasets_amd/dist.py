"""One process per GPU over RCCL (torch.distributed backend "nccl" == RCCL on ROCm).

Replaces the reference's nn.DataParallel (trainers/coop.py:435-436, cocoop.py:308-311),
which re-broadcast all ~150M frozen CLIP weights every step and reduced the prompt
gradients onto GPU 0 (and is broken for these trainers at >1 GPU). Here
every rank loads the frozen weights once, processes its own images (data parallel,
weak scaling), and the only collective is ONE all-reduce of the flattened trainable
prompt gradients per step (ctx [+ meta_net]: 8K-77K fp32, latency-bound on xGMI).
"""
from __future__ import annotations

import os

import torch
import torch.distributed as td


def is_dist() -> bool:
    return td.is_available() and td.is_initialized()


def rank() -> int:
    return td.get_rank() if is_dist() else 0


def world_size() -> int:
    return td.get_world_size() if is_dist() else 1


def init_from_env(backend: str | None = None) -> int:
    """Initialise from torchrun env (RANK/WORLD_SIZE/MASTER_*). Returns local rank."""
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if ws > 1 and not is_dist():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(local)
            td.init_process_group(backend, device_id=torch.device("cuda", local))
        else:
            td.init_process_group(backend)
    return local


def allreduce_grads(params, average: bool = True):
    """Sum (mean) the gradients of ``params`` across ranks in ONE fused bucket."""
    if not is_dist() or world_size() == 1:
        return
    grads = [p.grad for p in params if p.grad is not None]
    if not grads:
        return
    flat = torch.cat([g.reshape(-1) for g in grads])
    td.all_reduce(flat, op=td.ReduceOp.SUM)
    if average:
        flat.div_(world_size())
    off = 0
    for g in grads:
        n = g.numel()
        g.copy_(flat[off:off + n].view_as(g))
        off += n


def broadcast_params(params, src: int = 0):
    """Make the trainable prompt parameters identical on every rank (one bucket)."""
    if not is_dist() or world_size() == 1:
        return
    ps = list(params)
    flat = torch.cat([p.detach().reshape(-1) for p in ps])
    td.broadcast(flat, src)
    off = 0
    with torch.no_grad():
        for p in ps:
            n = p.numel()
            p.copy_(flat[off:off + n].view_as(p))
            off += n


def shard_range(n: int, r: int | None = None, w: int | None = None):
    """Contiguous [lo, hi) share of n items for rank r of w (eval-set sharding)."""
    r = rank() if r is None else r
    w = world_size() if w is None else w
    base, rem = divmod(n, w)
    lo = r * base + min(r, rem)
    return lo, lo + base + (1 if r < rem else 0)


def barrier():
    if is_dist():
        td.barrier()


def max_over_ranks(x: float) -> float:
    if not is_dist():
        return x
    dev = torch.device("cuda", torch.cuda.current_device()) if td.get_backend() == "nccl" else torch.device("cpu")
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    td.all_reduce(t, op=td.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(x: float) -> float:
    if not is_dist():
        return x
    dev = torch.device("cuda", torch.cuda.current_device()) if td.get_backend() == "nccl" else torch.device("cpu")
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    td.all_reduce(t, op=td.ReduceOp.SUM)
    return float(t.item())
