"""CPU: the oracle (oracle/clip_oracle.py, fp32 torch restatement) against the golden
vectors the reference itself produced (tests/golden/make_golden.py). Pins the oracle.

Also pins the synthetic generators (weight digest recorded in every fixture) and the
truncation identity: the oracle at L = max EOT + 1 reproduces the 77-token reference.
"""
import numpy as np
import pytest
import torch

from oracle import clip_oracle as O
from parity_util import load_fixture, rel_err
from fsp_amd.clip import synth

TINY = ["coop_tiny_end_csc0_ce", "coop_tiny_end_csc1_ce", "coop_tiny_middle_csc0_ce",
        "coop_tiny_middle_csc1_ce", "coop_tiny_front_csc0_ce", "coop_tiny_front_csc1_ce",
        "coop_tiny_end_focal", "coop_tiny_end_simclr", "coop_tiny_ctxinit_ce", "coop_tinyp8_end_ce"]
FULL = ["coop_vitb32_c10", "coop_vitb16_c6_focal", "coop_vitl14_c4"]

_SD = {}


def sd_for(arch):
    if arch not in _SD:
        _SD.clear()
        _SD[arch] = synth.make_state_dict(arch, seed=0)
    return _SD[arch]


def coop_oracle(meta, ref, truncate):
    sd = sd_for(meta["arch"])
    assert synth.state_dict_digest(sd) == meta["digest"], "synthetic weight generator drifted"
    p = O.as_torch_sd(sd)
    a = synth.ARCHS[meta["arch"]]
    tok = torch.from_numpy(ref["tokenized"].astype(np.int64))
    emb = O.token_embed(p, tok)
    n_ctx = ref["ctx0"].shape[-2]
    prefix, suffix = emb[:, :1], emb[:, 1 + n_ctx:]
    ctx = torch.from_numpy(ref["ctx0"]).requires_grad_(True)
    img = torch.from_numpy(synth.make_images(meta["batch"], a.image_resolution, seed=1))
    L = int(tok.argmax(-1).max()) + 1 if truncate else None
    logits = O.coop_logits(p, img, ctx, prefix, suffix, tok, ref["name_lens"], meta["position"], L)
    if meta["loss_type"] == "simclr":
        img2 = torch.from_numpy(synth.make_images(meta["batch"], a.image_resolution, seed=5))
        l2 = O.coop_logits(p, img2, ctx, prefix, suffix, tok, ref["name_lens"], meta["position"], L)
        loss = O.ntxent_logits_loss(logits, l2)
    else:
        y = torch.from_numpy(synth.make_labels(meta["batch"], meta["n_cls"], seed=2))
        if meta["loss_type"] == "focal":
            shots = [4, 1, 2, 0, 3] if meta["arch"] == "tiny" else [16, 16, 16, 1, 1, 1]
            loss = O.focal_loss(logits, y, O.focal_alpha(shots, meta["n_cls"]))
        else:
            loss = torch.nn.functional.cross_entropy(logits, y)
    loss.backward()
    (p1,), _ = O.sgd_step([ctx.detach()], [ctx.grad], [None], 0.002)
    return logits.detach().numpy(), float(loss), ctx.grad.numpy(), p1.numpy()


@pytest.mark.parametrize("truncate", [False, True])
@pytest.mark.parametrize("name", TINY)
def test_oracle_coop_tiny(name, truncate):
    meta, ref = load_fixture(name)
    logits, loss, g, step = coop_oracle(meta, ref, truncate)
    assert np.abs(logits - ref["logits"]).max() <= 2e-5
    assert rel_err(loss, ref["loss"]) <= 1e-5
    assert rel_err(g, ref["grad_ctx"]) <= 1e-4
    assert rel_err(step, ref["ctx_after_step"]) <= 1e-5


@pytest.mark.parametrize("name", FULL)
def test_oracle_coop_full(name):
    meta, ref = load_fixture(name)
    torch.set_num_threads(8)
    logits, loss, g, step = coop_oracle(meta, ref, True)
    assert np.abs(logits - ref["logits"]).max() <= 1e-4
    assert rel_err(g, ref["grad_ctx"]) <= 1e-3


def cocoop_oracle(meta, ref, truncate=True):
    sd = sd_for(meta["arch"])
    assert synth.state_dict_digest(sd) == meta["digest"]
    p = O.as_torch_sd(sd)
    a = synth.ARCHS[meta["arch"]]
    mp = {k: torch.from_numpy(v).requires_grad_(True)
          for k, v in synth.make_meta_net(a.embed_dim, a.transformer_width, seed=4).items()}
    tok = torch.from_numpy(ref["tokenized"].astype(np.int64))
    emb = O.token_embed(p, tok)
    n_ctx = meta["n_ctx"]
    ctx = torch.from_numpy(ref["ctx0"]).requires_grad_(True)
    img = torch.from_numpy(synth.make_images(meta["batch"], a.image_resolution, seed=1))
    L = int(tok.argmax(-1).max()) + 1 if truncate else None
    logits = O.cocoop_logits(p, mp, img, ctx, emb[:, :1], emb[:, 1 + n_ctx:], tok, L)
    y = torch.from_numpy(synth.make_labels(meta["batch"], meta["n_cls"], seed=2))
    if meta["focal"]:
        loss = O.focal_loss(logits, y, O.focal_alpha([4, 1, 2, 5, 3], meta["n_cls"], zero_guard=False))
    else:
        loss = torch.nn.functional.cross_entropy(logits, y)
    loss.backward()
    grads = {"grad_ctx": ctx.grad.numpy()}
    grads.update({"grad_" + k: v.grad.numpy() for k, v in mp.items()})
    return logits.detach().numpy(), float(loss), grads


@pytest.mark.parametrize("name", ["cocoop_tiny_ctxinit_ce", "cocoop_tiny_focal", "cocoop_vitb16_c4",
                                  "cocoop_vitl14_336_c3"])
def test_oracle_cocoop(name):
    """Also at ViT-L/14@336px (577 image tokens, W = 768 text): the only reference output at the
    config-5 architecture, which pins the oracle that gates config 5 at C = 1,000."""
    meta, ref = load_fixture(name)
    torch.set_num_threads(8)
    logits, loss, grads = cocoop_oracle(meta, ref)
    assert np.abs(logits - ref["logits"]).max() <= 1e-4
    assert rel_err(loss, ref["loss"]) <= 1e-5
    for k, v in grads.items():
        assert rel_err(v, ref[k]) <= 1e-3, k


def test_lr_schedule_matches_dassl():
    from fsp_amd.engine.optim import warmup_cosine_lr
    import os
    z = np.load(os.path.join(os.path.dirname(__file__), "golden", "lr_schedule.npz"))
    for key, me in (("ep10", 10), ("ep50", 50)):
        mine = [warmup_cosine_lr(e, 0.002, me, 1, "constant", 1e-5) for e in range(me)]
        assert np.abs(np.asarray(mine) - z[key]).max() < 1e-12
        orc = [O.cosine_lr(e, 0.002, me) for e in range(me)]
        assert np.abs(np.asarray(orc) - z[key]).max() < 1e-12
