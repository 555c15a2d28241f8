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
  ``AllGatherRows``;
* CoCoOp with class sharding (SURVEY §8(e) Option B, the reference's batch-1 configs):
  every rank scores the same images against its C/W classes, one all-gather of the
  [B, C_r] logits (``GatherClassColumns``) and a SUM all-reduce of the prompt gradients.
Eval shards the test set and gathers (label, prediction) pairs -- ``all_gather_varlen``.
The uneven-shard pad / unpad (``pad_rank_blocks`` / ``unpad_rank_blocks``) is shared by the
RCCL and gloo branches; only the collective call itself differs.
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
    """Initialise from torchrun env (RANK/WORLD_SIZE/MASTER_*). Returns local rank. A
    1-rank torchrun launch (WORLD_SIZE=1 with RANK / MASTER_PORT) also forms a group, so every
    RCCL branch below runs (tests/test_dist_nccl_gpu.py); otherwise this stays a plain process."""
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    launched = ws > 1 or (ws == 1 and "RANK" in os.environ and "MASTER_PORT" in os.environ)
    if launched and not is_dist():
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


def _grad_bucket(ps):
    """The persistent flat buffer of a fixed parameter list and one view of it per parameter,
    kept on the first parameter (its lifetime) and rebuilt when the list or a shape changes."""
    sig = tuple((id(p), tuple(p.shape)) for p in ps) + (ps[0].grad.dtype, ps[0].grad.device)
    b = getattr(ps[0], "_clipk_grad_bucket", None)
    if b is None or b[0] != sig:
        flat = torch.empty(sum(p.numel() for p in ps), dtype=ps[0].grad.dtype, device=ps[0].grad.device)
        views, off = [], 0
        for p in ps:
            views.append(flat[off:off + p.numel()].view_as(p))
            off += p.numel()
        b = (sig, flat, views)
        ps[0]._clipk_grad_bucket = b
    return b[1], b[2]


def allreduce_grads(params, average: bool = True, optimizer=None):
    """Sum (mean) the gradients of ``params`` across ranks in ONE fused bucket: the gradients are
    copied into a persistent flat buffer (one multi-tensor copy, or none when they already are its
    views), reduced in place, and each ``p.grad`` is rebound to its view of the result (no
    per-step concatenation, no copy back). ``optimizer`` with ``defer_grad_scale`` (FusedSGD):
    the mean's 1 / world is folded into its next step (clipk_sgd_step_multi_scaled) instead of a
    division launch -- the grads then hold the SUM, tagged with the pending scale, until that step
    (a step skipped by the amp finite check leaves the tag to the next all-reduce, which resets it)."""
    if not is_dist():
        return
    ps = [p for p in params if p.grad is not None]
    if not ps:
        return
    if len({(p.grad.dtype, p.grad.device) for p in ps}) != 1:
        raise ValueError("allreduce_grads: the gradients of one bucket must share dtype and device")
    flat, views = _grad_bucket(ps)
    todo = [(v, p.grad) for p, v in zip(ps, views) if p.grad.data_ptr() != v.data_ptr()]
    if todo:
        torch._foreach_copy_([v for v, _ in todo], [g for _, g in todo])
    _all_reduce(flat)
    if average and world_size() > 1:
        if optimizer is not None and hasattr(optimizer, "defer_grad_scale"):
            optimizer.defer_grad_scale(views, 1.0 / world_size())
        else:
            flat.div_(world_size())
    for p, v in zip(ps, views):
        p.grad = v


def broadcast_params(params, src: int = 0):
    """Make the trainable prompt parameters identical on every rank (one bucket)."""
    if not is_dist():
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


def batches_replicated(cfg) -> bool:
    """True when every rank must see the SAME batches and test images: CoCoOp with class
    sharding (cfg NATIVE.COCOOP_SHARD "class") at world > 1. Otherwise batches are split over
    the ranks (data parallel)."""
    nat = cfg.get("NATIVE", {}) or {}
    return (world_size() > 1 and str(cfg.TRAINER.get("NAME", "")) == "CoCoOp"
            and nat.get("COCOOP_SHARD", "image") == "class")


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
    if not is_dist():
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


def pad_rank_blocks(x, counts):
    """Rows [sum(counts), ...] in rank order -> [w * m, ...] (m = max(counts)) with rank i's
    rows at block i and zero padding after them: the equal-size layout that all-gather /
    reduce-scatter of uneven row shards need."""
    w, m = len(counts), max(counts)
    x = x.contiguous()
    if x.shape[0] != sum(counts):
        raise ValueError(f"{x.shape[0]} rows for shard counts {counts}")
    out = torch.zeros((w * m,) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    off = 0
    for i, k in enumerate(counts):
        out[i * m:i * m + k] = x[off:off + k]
        off += k
    return out


def unpad_rank_blocks(padded, counts):
    """Inverse of pad_rank_blocks: [w * m, ...] blocks -> rows [sum(counts), ...]."""
    m = max(counts)
    return torch.cat([padded[i * m:i * m + k] for i, k in enumerate(counts)], 0)


def reduce_scatter_rows(g, counts):
    """Sum ``g`` [sum(counts), ...] over ranks; return this rank's rows (counts[rank]).
    RCCL: reduce_scatter_tensor on the padded blocks; gloo (no reduce-scatter): the same
    padded blocks all-reduced on the host, then this rank's block."""
    r = rank()
    m = max(counts)
    if g.shape[0] != sum(counts):
        raise ValueError(f"{g.shape[0]} rows for shard counts {counts}")
    padded = g.contiguous() if min(counts) == m else pad_rank_blocks(g, counts)
    if td.get_backend() == "nccl":
        out = torch.empty((m,) + tuple(g.shape[1:]), dtype=g.dtype, device=g.device)
        td.reduce_scatter_tensor(out, padded, op=td.ReduceOp.SUM)
    else:
        out = _all_reduce(padded)[r * m:(r + 1) * m]
    return out[:counts[r]].contiguous()


def all_gather_rows(x, counts):
    """Every rank's row block [counts[r], ...] -> [sum(counts), ...] on every rank (rank
    order), through equal-size padded blocks (all_gather_into_tensor on RCCL); equal shards
    (C divisible by the world size) skip the padding and unpadding copies."""
    w, m = len(counts), max(counts)
    xc = x.contiguous()
    if min(counts) == m:
        h = _host(xc)
        if td.get_backend() == "nccl":
            full = torch.empty((w * m,) + tuple(h.shape[1:]), dtype=h.dtype, device=h.device)
            td.all_gather_into_tensor(full, h)
        else:
            parts = [torch.empty_like(h) for _ in range(w)]
            td.all_gather(parts, h)
            full = torch.cat(parts, 0)
        return full.to(x.device)
    pad = torch.zeros((m,) + tuple(xc.shape[1:]), dtype=xc.dtype, device=xc.device)
    pad[:xc.shape[0]] = xc
    h = _host(pad)
    if td.get_backend() == "nccl":
        full = torch.empty((w * m,) + tuple(h.shape[1:]), dtype=h.dtype, device=h.device)
        td.all_gather_into_tensor(full, h)
    else:
        parts = [torch.empty_like(h) for _ in range(w)]
        td.all_gather(parts, h)
        full = torch.cat(parts, 0)
    return unpad_rank_blocks(full, counts).to(x.device)


class AllGatherRows(torch.autograd.Function):
    """Forward: every rank's row block [n_r, E] -> the full [sum n_r, E] on every rank
    (rank order). Backward: each rank's dL_r/d(full) is summed over ranks and the owner
    keeps its rows (reduce_scatter_rows). CoOp class-sharded text features: rank r encodes
    classes [lo_r, hi_r) (shard_range) and every rank forms the logits of ITS images against
    all C classes; the owner backpropagates the summed text-feature gradient through its own
    slice of the text encoder."""

    @staticmethod
    def forward(ctx, x, counts):
        ctx.counts = counts
        return all_gather_rows(x, counts)

    @staticmethod
    def backward(ctx, g):
        return reduce_scatter_rows(g, ctx.counts), None


class GatherClassColumns(torch.autograd.Function):
    """CoCoOp class sharding (SURVEY §8(e) Option B): rank r holds the logits [B, C_r] of
    its classes for the SAME B images as every other rank; forward all-gathers them into
    [B, C] (class order = rank order). Every rank then evaluates the identical full loss, so
    dL/d(logits) is the same on every rank and the backward only slices out this rank's
    columns -- no collective. The prompt gradients each rank produces are partial sums over
    its classes: all-reduce them with SUM (allreduce_grads(average=False))."""

    @staticmethod
    def forward(ctx, x, counts):
        ctx.counts = counts
        ctx.r = rank()
        w = len(counts)
        if min(counts) == max(counts) and td.get_backend() == "nccl":
            # equal shards: gather the [B, C_r] blocks as they are and interleave them into
            # [B, C] with one copy (no transposes, no padding)
            xc = x.contiguous()
            buf = torch.empty((w,) + tuple(xc.shape), dtype=xc.dtype, device=xc.device)
            td.all_gather_into_tensor(buf, xc)
            return buf.permute(1, 0, 2).reshape(xc.shape[0], w * xc.shape[1])
        full_t = all_gather_rows(x.t(), counts)  # [C, B]
        return full_t.t().contiguous()

    @staticmethod
    def backward(ctx, g):
        lo = sum(ctx.counts[:ctx.r])
        return g[:, lo:lo + ctx.counts[ctx.r]].contiguous(), None


def sync_rng_from(src: int = 0):
    """Make torch's CPU RNG state identical on every rank (rank ``src``'s), so samplers that
    draw from the global generator (RandomSampler, WeightedRandomSampler, as the reference's
    DataManager builds them) produce the same global index stream on every rank."""
    if not is_dist():
        return
    st = torch.get_rng_state()
    if td.get_backend() == "nccl":
        st = st.to(torch.device("cuda", torch.cuda.current_device()))
    td.broadcast(st, src)
    torch.set_rng_state(st.cpu())


def broadcast_int(v: int, src: int = 0) -> int:
    """Rank ``src``'s integer on every rank (e.g. a seed)."""
    if not is_dist():
        return int(v)
    dev = torch.device("cuda", torch.cuda.current_device()) if td.get_backend() == "nccl" else torch.device("cpu")
    t = torch.tensor([int(v)], dtype=torch.int64, device=dev)
    td.broadcast(t, src)
    return int(t.item())


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
