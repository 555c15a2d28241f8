"""One process per GPU over RCCL (torch.distributed backend "nccl" == RCCL on ROCm).

Replaces the reference's nn.DataParallel (trainers/coop.py:435-436, cocoop.py:308-311),
which re-broadcast all ~150M frozen CLIP weights every step and reduced the prompt
gradients onto GPU 0 (and is broken for these trainers at >1 GPU). Here
every rank loads the frozen weights once and processes its own images (data parallel);
per step the collectives are:
* ONE all-reduce of the flattened trainable prompt gradients (ctx [+ meta_net]: 8K-77K
  fp32, latency-bound on xGMI) -- ``allreduce_grads``;
* CoOp with class-sharded text encoding: an all-gather of the [C, E] text
  features and, in backward, a reduce-scatter of dL/dtext to the class owners --
  ``AllGatherRows``.
Eval shards the test set and gathers (label, prediction) pairs -- ``all_gather_varlen``.
With the gloo backend (CPU tests, or several ranks sharing one GPU) CUDA tensors go through
host copies.
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


def _host(t):
    """gloo collectives on CUDA tensors: run them on a host copy."""
    return t.cpu() if (t.is_cuda and td.get_backend() == "gloo") else t


def _all_reduce(t, op=td.ReduceOp.SUM):
    h = _host(t)
    td.all_reduce(h, op=op)
    if h is not t:
        t.copy_(h)
    return t


def allreduce_grads(params, average: bool = True):
    """Sum (mean) the gradients of ``params`` across ranks in ONE fused bucket."""
    if not is_dist() or world_size() == 1:
        return
    grads = [p.grad for p in params if p.grad is not None]
    if not grads:
        return
    flat = torch.cat([g.reshape(-1) for g in grads])
    _all_reduce(flat)
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
    h = _host(flat)
    td.broadcast(h, src)
    if h is not flat:
        flat.copy_(h)
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


def all_gather_varlen(t):
    """Concatenate every rank's ``t`` (same trailing shape, any leading length) in rank
    order; returned on every rank, on t's device."""
    if not is_dist() or world_size() == 1:
        return t
    w = world_size()
    h = _host(t.contiguous())
    n = torch.tensor([h.shape[0]], dtype=torch.int64, device=h.device)
    ns = [torch.zeros_like(n) for _ in range(w)]
    td.all_gather(ns, n)
    ns = [int(x.item()) for x in ns]
    m = max(ns)
    pad = torch.zeros((m,) + tuple(h.shape[1:]), dtype=h.dtype, device=h.device)
    pad[:h.shape[0]] = h
    parts = [torch.empty_like(pad) for _ in range(w)]
    td.all_gather(parts, pad)
    out = torch.cat([p[:k] for p, k in zip(parts, ns)], 0)
    return out.to(t.device)


class AllGatherRows(torch.autograd.Function):
    """Forward: every rank's row block [n_r, E] -> the full [sum n_r, E] on every rank
    (rank order). Backward: each rank's dL_r/d(full) is summed over ranks and the owner
    keeps its rows (a reduce-scatter; all-reduce + slice on gloo). CoOp class-sharded text
    features: rank r encodes classes [lo_r, hi_r) (shard_range) and every rank forms the
    logits against all C classes; the owner backpropagates the summed text-feature gradient
    through its own slice of the text encoder."""

    @staticmethod
    def forward(ctx, x, counts):
        ctx.counts = counts
        ctx.r = rank()
        w = len(counts)
        m = max(counts)
        xc = x.contiguous()
        pad = torch.zeros((m,) + tuple(xc.shape[1:]), dtype=xc.dtype, device=xc.device)
        pad[:xc.shape[0]] = xc
        h = _host(pad)
        parts = [torch.empty_like(h) for _ in range(w)]
        td.all_gather(parts, h)
        return torch.cat([p[:k] for p, k in zip(parts, counts)], 0).to(x.device)

    @staticmethod
    def backward(ctx, g):
        counts, r = ctx.counts, ctx.r
        lo = sum(counts[:r])
        g = g.contiguous()
        if td.get_backend() == "nccl":
            w, m = len(counts), max(counts)
            padded = torch.zeros((w * m,) + tuple(g.shape[1:]), dtype=g.dtype, device=g.device)
            off = 0
            for i, k in enumerate(counts):
                padded[i * m:i * m + k] = g[off:off + k]
                off += k
            out = torch.empty((m,) + tuple(g.shape[1:]), dtype=g.dtype, device=g.device)
            td.reduce_scatter_tensor(out, padded, op=td.ReduceOp.SUM)
            return out[:counts[r]], None
        full = _all_reduce(g.clone())
        return full[lo:lo + counts[r]].contiguous(), None


def sync_rng_from(src: int = 0):
    """Make torch's CPU RNG state identical on every rank (rank ``src``'s), so samplers that
    draw from the global generator (RandomSampler, WeightedRandomSampler, as the reference's
    DataManager builds them) produce the same global index stream on every rank."""
    if not is_dist() or world_size() == 1:
        return
    st = torch.get_rng_state()
    if td.get_backend() == "nccl":
        st = st.to(torch.device("cuda", torch.cuda.current_device()))
    td.broadcast(st, src)
    torch.set_rng_state(st.cpu())


def barrier():
    if is_dist():
        td.barrier()


def max_over_ranks(x: float) -> float:
    if not is_dist():
        return x
    dev = torch.device("cuda", torch.cuda.current_device()) if td.get_backend() == "nccl" else torch.device("cpu")
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    _all_reduce(t, op=td.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(x: float) -> float:
    if not is_dist():
        return x
    dev = torch.device("cuda", torch.cuda.current_device()) if td.get_backend() == "nccl" else torch.device("cpu")
    t = torch.tensor([x], dtype=torch.float64, device=dev)
    _all_reduce(t)
    return float(t.item())
