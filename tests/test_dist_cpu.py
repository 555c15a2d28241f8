"""CPU, world_size 2 over gloo: the multi-process data-parallel path (fsp_amd.dist).

Checks the collective helpers and the DP semantics the trainers rely on: each rank
backprops its own images, one fused all-reduce averages the prompt gradients, and the
result equals the gradient of the mean loss over the union batch (the oracle supplies
the per-rank CoCoOp gradients on CPU)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, fn, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from fsp_amd import dist
    dist.init_from_env(backend="gloo")
    try:
        q.put((rank, fn(rank, world)))
    finally:
        torch.distributed.destroy_process_group()


def _run(fn, world=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, fn, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return out


def _collectives(rank, world):
    from fsp_amd import dist
    p1 = torch.nn.Parameter(torch.full((3, 4), float(rank + 1)))
    p2 = torch.nn.Parameter(torch.zeros(5))
    p1.grad = torch.full((3, 4), float(rank + 1))
    p2.grad = torch.arange(5, dtype=torch.float32) * (rank + 1)
    dist.allreduce_grads([p1, p2])
    dist.broadcast_params([p1, p2], src=1)
    return {
        "g1": p1.grad.clone().numpy(), "g2": p2.grad.clone().numpy(), "p1": p1.detach().numpy().copy(),
        "shard": dist.shard_range(10), "max": dist.max_over_ranks(float(rank)),
        "sum": dist.sum_over_ranks(float(rank + 1)), "ws": dist.world_size(),
    }


def test_collectives_gloo_ws2():
    out = _run(_collectives)
    for r in (0, 1):
        np.testing.assert_allclose(out[r]["g1"], np.full((3, 4), 1.5))
        np.testing.assert_allclose(out[r]["g2"], np.arange(5) * 1.5)
        np.testing.assert_allclose(out[r]["p1"], np.full((3, 4), 2.0))  # broadcast from rank 1
        assert out[r]["max"] == 1.0 and out[r]["sum"] == 3.0 and out[r]["ws"] == 2
    assert out[0]["shard"] == (0, 5) and out[1]["shard"] == (5, 10)


def _cocoop_dp(rank, world):
    """Per-rank CoCoOp grads on its half of the batch (oracle math), then dist.allreduce."""
    from oracle import clip_oracle as O
    from fsp_amd.clip import synth
    from fsp_amd import dist
    from parity_util import load_fixture
    meta, ref = load_fixture("cocoop_tiny_ctxinit_ce")
    a = synth.ARCHS["tiny"]
    p = O.as_torch_sd(synth.make_state_dict("tiny", seed=0))
    mp_ = {k: torch.nn.Parameter(torch.from_numpy(v)) for k, v in
           synth.make_meta_net(a.embed_dim, a.transformer_width, seed=4).items()}
    tok = torch.from_numpy(ref["tokenized"].astype(np.int64))
    emb = O.token_embed(p, tok)
    ctx = torch.nn.Parameter(torch.from_numpy(ref["ctx0"]))
    img = torch.from_numpy(synth.make_images(4, a.image_resolution, seed=1))
    y = torch.from_numpy(synth.make_labels(4, meta["n_cls"], seed=2))
    lo, hi = dist.shard_range(4)
    logits = O.cocoop_logits(p, mp_, img[lo:hi], ctx, emb[:, :1], emb[:, 1 + 4:], tok)
    torch.nn.functional.cross_entropy(logits, y[lo:hi]).backward()
    params = [ctx] + list(mp_.values())
    dist.allreduce_grads(params)
    return {"ctx": ctx.grad.numpy().copy(), "w1": mp_["meta_net.linear1.weight"].grad.numpy().copy()}


def test_data_parallel_grad_equals_full_batch():
    out = _run(_cocoop_dp)
    from oracle import clip_oracle as O
    from fsp_amd.clip import synth
    from parity_util import load_fixture
    meta, ref = load_fixture("cocoop_tiny_ctxinit_ce")
    a = synth.ARCHS["tiny"]
    p = O.as_torch_sd(synth.make_state_dict("tiny", seed=0))
    mp_ = {k: torch.nn.Parameter(torch.from_numpy(v)) for k, v in
           synth.make_meta_net(a.embed_dim, a.transformer_width, seed=4).items()}
    tok = torch.from_numpy(ref["tokenized"].astype(np.int64))
    emb = O.token_embed(p, tok)
    ctx = torch.nn.Parameter(torch.from_numpy(ref["ctx0"]))
    img = torch.from_numpy(synth.make_images(4, a.image_resolution, seed=1))
    y = torch.from_numpy(synth.make_labels(4, meta["n_cls"], seed=2))
    logits = O.cocoop_logits(p, mp_, img, ctx, emb[:, :1], emb[:, 1 + 4:], tok)
    torch.nn.functional.cross_entropy(logits, y).backward()
    for r in (0, 1):
        np.testing.assert_allclose(out[r]["ctx"], ctx.grad.numpy(), rtol=1e-4, atol=2e-6)
        np.testing.assert_allclose(out[r]["w1"], mp_["meta_net.linear1.weight"].grad.numpy(), rtol=1e-4, atol=2e-6)
