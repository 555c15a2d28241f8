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


def _grad_allreduce_timer(rank, world):
    import bench
    p1 = torch.nn.Parameter(torch.ones(3, 4))
    p2 = torch.nn.Parameter(torch.ones(5))
    frozen = torch.nn.Parameter(torch.ones(2), requires_grad=False)
    r = bench.time_grad_allreduce([p1, p2, frozen], iters=3, warmup=1)
    return r, p1.grad.clone().numpy()


def test_bench_grad_allreduce_timer_gloo_ws2():
    """bench.py's N > 1 field grad_allreduce: the trainable parameters' bytes, a positive time
    equal on every rank (max over ranks), the collective really summing (zeros in, zeros out)."""
    out = _run(_grad_allreduce_timer)
    for rk in (0, 1):
        r, g = out[rk]
        assert r["bytes"] == 4 * 17 and r["iters"] == 3 and r["backend"] == "gloo" and r["us_per_call"] > 0
        np.testing.assert_array_equal(g, np.zeros((3, 4)))
    assert out[0][0]["us_per_call"] == out[1][0]["us_per_call"]


def _bucket_steps(rank, world):
    """Three steps through one persistent gradient bucket: fresh grads (zero_grad to None), then
    grads accumulated in place into the bucket's views (zero_grad(set_to_none=False))."""
    from fsp_amd import dist
    p1 = torch.nn.Parameter(torch.zeros(3, 4))
    p2 = torch.nn.Parameter(torch.zeros(5))
    opt = torch.optim.SGD([p1, p2], lr=0.1)
    out = []
    for step, none in enumerate((True, True, False)):
        opt.zero_grad(set_to_none=none)
        ((p1 * (rank + 1 + step)).sum() + (p2 * torch.arange(5.0) * (rank + 1)).sum()).backward()
        dist.allreduce_grads([p1, p2])
        out.append((p1.grad.clone().numpy(), p2.grad.clone().numpy(),
                    p1.grad.data_ptr() == p1._clipk_grad_bucket[1].data_ptr()))
    return out


def test_grad_bucket_persists_across_steps():
    out = _run(_bucket_steps)
    for r in (0, 1):
        for step, (g1, g2, rebound) in enumerate(out[r]):
            np.testing.assert_allclose(g1, np.full((3, 4), 1.5 + step))  # mean of rank+1+step
            np.testing.assert_allclose(g2, np.arange(5) * 1.5)
            assert rebound


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


def _sampler_shards(rank, world):
    """Every rank walks the same global sampler stream (RNG synced from rank 0) and takes
    its slice of each global batch."""
    from fsp_amd import dist
    from fsp_amd.data.fewshot import Datum, WeightedClassSampler
    from fsp_amd.data.manager import ShardedBatchSampler
    from torch.utils.data import RandomSampler
    torch.manual_seed(1234 + 7 * rank)  # ranks start out of sync on purpose
    data = [Datum(impath=f"x{i}", label=i % 4 if i < 14 else 0) for i in range(23)]
    out = {}
    for name, smp in (("random", RandomSampler(data)), ("weighted", WeightedClassSampler(data))):
        dist.sync_rng_from(0)
        bs = ShardedBatchSampler(smp, batch_size=3, drop_last=False)
        out[name] = [list(b) for b in bs]
        out[name + "_len"] = len(bs)
    return out


def test_sharded_batches_union_is_the_global_stream():
    out = _run(_sampler_shards)
    from fsp_amd.data.fewshot import Datum, WeightedClassSampler
    from torch.utils.data import RandomSampler
    data = [Datum(impath=f"x{i}", label=i % 4 if i < 14 else 0) for i in range(23)]
    for name, cls in (("random", RandomSampler), ("weighted", WeightedClassSampler)):
        torch.manual_seed(1234)  # rank 0's state, which every rank adopted
        if name == "weighted":
            list(RandomSampler(data))  # rank 0 consumed the random stream first
        glob = list(iter(cls(data)))
        batches = [glob[b:b + 6] for b in range(0, len(glob), 6)]
        assert out[0][name + "_len"] == out[1][name + "_len"] == len(batches)
        for i, gb in enumerate(batches):
            k0, k1 = out[0][name][i], out[1][name][i]
            assert all(n == len(gb) for _, n, _ in k0 + k1)  # n_global rides along
            got = [j for j, _, _ in k0] + [j for j, _, _ in k1]
            if len(gb) >= 2:
                assert got == gb
                assert [nl for _, _, nl in k0 + k1] == [len(k0)] * len(k0) + [len(k1)] * len(k1)
            else:  # a 1-item last batch: rank 1 gets it as a pad (local size 0, loss weight 0)
                assert got == gb + gb
                assert k0[0][2] == 1 and k1[0][2] == 0


def _test_sharded_eval(rank, world):
    """TrainerX.test on each rank's contiguous shard of the test set (test double model on
    CPU): every rank returns the labels / predictions / accuracy of the WHOLE set."""
    import tempfile
    from fsp_amd import dist
    from test_host_cpu import _dummy_trainer
    rs = np.random.RandomState(3)
    imgs = torch.from_numpy(rs.randn(23, 3, 2, 2).astype(np.float32))
    lbl = torch.from_numpy(rs.randint(0, 3, 23))
    lo, hi = dist.shard_range(23)
    mine = [{"img": imgs[i:min(i + 5, hi)], "label": lbl[i:min(i + 5, hi)]} for i in range(lo, hi, 5)]
    t = _dummy_trainer(tempfile.mkdtemp(), mine)
    y_true, y_pred = t.test(return_pred=True)
    return {"y_true": y_true, "y_pred": y_pred, "acc": t.test()}


def test_eval_sharded_over_ranks_matches_single_process(tmp_path):
    out = _run(_test_sharded_eval)
    from test_host_cpu import _dummy_trainer
    rs = np.random.RandomState(3)
    imgs = torch.from_numpy(rs.randn(23, 3, 2, 2).astype(np.float32))
    lbl = torch.from_numpy(rs.randint(0, 3, 23))
    t = _dummy_trainer(tmp_path, [{"img": imgs[i:i + 7], "label": lbl[i:i + 7]} for i in range(0, 23, 7)])
    y_true, y_pred = t.test(return_pred=True)
    acc = t.test()
    for r in (0, 1):
        np.testing.assert_array_equal(out[r]["y_true"], y_true)
        np.testing.assert_array_equal(out[r]["y_pred"], y_pred)
        assert out[r]["acc"] == acc


def _coop_sharded_grad(rank, world, n_img=5):
    """CoOp with class-sharded text encoding + image data parallel, on the oracle's math:
    rank r encodes classes shard_range(C) only, dist.AllGatherRows forms the [C, E] text
    features (reduce-scatter of their gradient in backward), each rank scores its own images
    (uneven 3 / 2 split) with the loss weighted by its batch share, then the averaged
    all-reduce of d ctx."""
    from oracle import clip_oracle as O
    from fsp_amd.clip import synth
    from fsp_amd import dist
    from fsp_amd.engine.trainer import TrainerX
    from parity_util import load_fixture
    meta, ref = load_fixture("coop_tiny_end_csc0_ce")
    p = O.as_torch_sd(synth.make_state_dict("tiny", seed=0))
    tok = torch.from_numpy(ref["tokenized"].astype(np.int64))
    emb = O.token_embed(p, tok)
    C = meta["n_cls"]
    counts = [hi - lo for lo, hi in (dist.shard_range(C, r, world) for r in range(world))]
    clo, chi = dist.shard_range(C)
    ctx = torch.nn.Parameter(torch.from_numpy(ref["ctx0"]))
    a = synth.ARCHS["tiny"]
    img = torch.from_numpy(synth.make_images(n_img, a.image_resolution, seed=1))
    y = torch.from_numpy(synth.make_labels(n_img, C, seed=2))
    ilo, ihi = dist.shard_range(n_img)
    pr = O.coop_prompts(ctx, emb[clo:chi, :1], emb[clo:chi, 5:], ref["name_lens"][clo:chi], "end")
    txt = dist.AllGatherRows.apply(O.encode_text(p, pr, tok[clo:chi]), counts)
    imf = O.normalize(O.encode_image(p, img[ilo:ihi]))
    logits = p["logit_scale"].exp() * imf @ O.normalize(txt).t()
    loss = torch.nn.functional.cross_entropy(logits, y[ilo:ihi])
    w = TrainerX.batch_weight({"n_global": n_img}, ihi - ilo)
    (loss * w).backward()
    dist.allreduce_grads([ctx])
    return {"ctx": ctx.grad.numpy().copy(), "txt": txt.detach().numpy().copy()}


def test_coop_class_sharded_grad_equals_full_batch():
    out = _run(_coop_sharded_grad)
    from oracle import clip_oracle as O
    from fsp_amd.clip import synth
    from parity_util import load_fixture
    meta, ref = load_fixture("coop_tiny_end_csc0_ce")
    p = O.as_torch_sd(synth.make_state_dict("tiny", seed=0))
    tok = torch.from_numpy(ref["tokenized"].astype(np.int64))
    emb = O.token_embed(p, tok)
    ctx = torch.nn.Parameter(torch.from_numpy(ref["ctx0"]))
    a = synth.ARCHS["tiny"]
    img = torch.from_numpy(synth.make_images(5, a.image_resolution, seed=1))
    y = torch.from_numpy(synth.make_labels(5, meta["n_cls"], seed=2))
    logits = O.coop_logits(p, img, ctx, emb[:, :1], emb[:, 5:], tok, ref["name_lens"], "end")
    torch.nn.functional.cross_entropy(logits, y).backward()
    txt = O.encode_text(p, O.coop_prompts(ctx.detach(), emb[:, :1], emb[:, 5:], ref["name_lens"], "end"), tok)
    for r in (0, 1):
        np.testing.assert_allclose(out[r]["txt"], txt.numpy(), rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(out[r]["ctx"], ctx.grad.numpy(), rtol=1e-4, atol=2e-5)


def test_pad_batch_has_zero_loss_weight():
    """The pad a rank receives when its slice of a short last batch is empty carries
    n_local 0: TrainerX.batch_weight gives it weight 0 (it joins the all-reduce with a zero
    gradient instead of counting the item twice)."""
    from fsp_amd.engine.trainer import TrainerX
    import fsp_amd.dist as D
    orig = D.world_size
    D.world_size = lambda: 2
    try:
        assert TrainerX.batch_weight({"n_global": 1, "n_local": 0}, 1) == 0.0
        assert TrainerX.batch_weight({"n_global": 1, "n_local": 1}, 1) == 2.0
        assert TrainerX.batch_weight({"n_global": 5, "n_local": 3}, 3) == 1.2
    finally:
        D.world_size = orig


def _rank_blocks(rank, world):
    """pad / unpad of uneven row shards (shared by the RCCL and gloo branches), the gloo
    reduce-scatter and all-gather built on them."""
    from fsp_amd import dist
    counts = [3, 2]
    g = torch.arange(5 * 2, dtype=torch.float32).reshape(5, 2) * (rank + 1)
    padded = dist.pad_rank_blocks(g, counts)
    back = dist.unpad_rank_blocks(padded, counts)
    mine = torch.full((counts[rank], 2), float(rank + 1))
    # equal shards take the no-padding path
    g4 = torch.arange(4 * 2, dtype=torch.float32).reshape(4, 2) * (rank + 1)
    mine2 = torch.full((2, 2), float(rank + 1))
    return {"padded": padded.numpy(), "back": back.numpy(), "rs": dist.reduce_scatter_rows(g, counts).numpy(),
            "ag": dist.all_gather_rows(mine, counts).numpy(),
            "rs_eq": dist.reduce_scatter_rows(g4, [2, 2]).numpy(), "ag_eq": dist.all_gather_rows(mine2, [2, 2]).numpy()}


def test_pad_reduce_scatter_all_gather_rows():
    out = _run(_rank_blocks)
    g = np.arange(10, dtype=np.float32).reshape(5, 2)
    for r in (0, 1):
        o = out[r]
        exp_pad = np.zeros((6, 2), np.float32)
        exp_pad[:3] = g[:3] * (r + 1)
        exp_pad[3:5] = g[3:] * (r + 1)
        np.testing.assert_array_equal(o["padded"], exp_pad)
        np.testing.assert_array_equal(o["back"], g * (r + 1))
        np.testing.assert_array_equal(o["rs"], (g * 3)[:3] if r == 0 else (g * 3)[3:])
        np.testing.assert_array_equal(o["ag"], np.array([[1, 1]] * 3 + [[2, 2]] * 2, np.float32))
        g4 = np.arange(8, dtype=np.float32).reshape(4, 2)
        np.testing.assert_array_equal(o["rs_eq"], (g4 * 3)[2 * r:2 * r + 2])
        np.testing.assert_array_equal(o["ag_eq"], np.array([[1, 1]] * 2 + [[2, 2]] * 2, np.float32))


def _augment_streams(rank, world):
    from fsp_amd.data.manager import augment_generator
    from fsp_amd.data.preprocess import train_plan
    torch.manual_seed(99 + rank)  # ranks' own seeds differ; rank 0's is the base
    out = {}
    for rep in (False, True):
        g = augment_generator(rep)
        out[rep] = [vars(train_plan(500, 375, 224, generator=g)) for _ in range(6)]
    return out


def test_augmentation_stream_per_rank():
    """Data parallel: each rank draws its own crop / flip stream (different crops for its
    different images); replicated batches (CoCoOp class sharding): one stream on every rank."""
    out = _run(_augment_streams)
    assert out[0][False] != out[1][False]
    assert out[0][True] == out[1][True]


def _cocoop_class_sharded(rank, world, n_img=1):
    """CoCoOp class sharding (Option B) on the oracle's math: every rank scores the SAME
    image(s) against its classes, GatherClassColumns forms the [B, C] logits, every rank
    evaluates the full CE, the partial prompt gradients are SUM all-reduced."""
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
    C = meta["n_cls"]
    counts = [hi - lo for lo, hi in (dist.shard_range(C, r, world) for r in range(world))]
    lo, hi = dist.shard_range(C)
    ctx = torch.nn.Parameter(torch.from_numpy(ref["ctx0"]))
    img = torch.from_numpy(synth.make_images(n_img, a.image_resolution, seed=1))
    y = torch.from_numpy(synth.make_labels(n_img, C, seed=2))
    local = O.cocoop_logits(p, mp_, img, ctx, emb[lo:hi, :1], emb[lo:hi, 1 + 4:], tok[lo:hi])
    logits = dist.GatherClassColumns.apply(local, counts)
    torch.nn.functional.cross_entropy(logits, y).backward()
    params = [ctx] + list(mp_.values())
    dist.allreduce_grads(params, average=False)
    return {"logits": logits.detach().numpy().copy(), "ctx": ctx.grad.numpy().copy(),
            "w1": mp_["meta_net.linear1.weight"].grad.numpy().copy()}


@pytest.mark.parametrize("n_img", [1, 2])
def test_cocoop_class_sharded_grad_equals_single_process(n_img):
    import functools
    out = _run(functools.partial(_cocoop_class_sharded, n_img=n_img))
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
    img = torch.from_numpy(synth.make_images(n_img, a.image_resolution, seed=1))
    y = torch.from_numpy(synth.make_labels(n_img, meta["n_cls"], seed=2))
    logits = O.cocoop_logits(p, mp_, img, ctx, emb[:, :1], emb[:, 1 + 4:], tok)
    torch.nn.functional.cross_entropy(logits, y).backward()
    for r in (0, 1):
        np.testing.assert_allclose(out[r]["logits"], logits.detach().numpy(), rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(out[r]["ctx"], ctx.grad.numpy(), rtol=1e-4, atol=2e-6)
        np.testing.assert_allclose(out[r]["w1"], mp_["meta_net.linear1.weight"].grad.numpy(), rtol=1e-4, atol=2e-6)


def _best_val_ranks(directory, rank, world):
    """TEST.FINAL_MODEL "best_val" with 2 ranks sharing OUTPUT_DIR: rank 0 alone writes
    model-best.pth.tar (and writes it slowly here); every rank must load the best-val weights
    it wrote -- never a missing, partial or older file -- before the final test."""
    import time
    from test_host_cpu import _dummy_trainer
    rs = np.random.RandomState(3)
    batches = [{"img": torch.from_numpy(rs.randn(5, 3, 2, 2).astype(np.float32)),
                "label": torch.from_numpy(rs.randint(0, 3, 5))} for _ in range(2)]
    t = _dummy_trainer(directory, batches)
    t.dm.val_loader = batches[:1]
    t.cfg.TEST.NO_TEST = False
    t.cfg.TEST.FINAL_MODEL = "best_val"
    vals = iter([10.0, 30.0, 20.0])
    tests = []
    orig_test, orig_save = t.test, t.save_model

    def fake_test(split=None, return_pred=False):
        if split == "val":
            return next(vals)
        tests.append(float(t.learner.ctx.detach()[0, 0]))
        return orig_test(split, return_pred)

    def slow_save(*a, **k):
        if rank == 0:  # the writer lags behind the other rank
            time.sleep(0.5)
        return orig_save(*a, **k)
    t.test = fake_test
    t.save_model = slow_save
    t.run_epoch = lambda: t.learner.ctx.data.add_(1.0)  # epoch e leaves ctx == e + 1
    t.train(start_epoch=0, max_epoch=3)
    return tests


def test_best_val_final_model_two_ranks(tmp_path):
    import functools
    out = _run(functools.partial(_best_val_ranks, str(tmp_path)))
    assert out[0] == [2.0] and out[1] == [2.0]  # both ranks test the 2nd epoch's (best) weights
