"""Helpers shared by the parity tests: load a golden fixture, rebuild the same model
and inputs with the native path, run the reference's forward/backward/step sequence."""
from __future__ import annotations

import json
import os

import numpy as np
import torch

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

_SD_CACHE = {}


def load_fixture(name):
    z = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    meta = json.loads(str(z["meta"]))
    arrays = {k: z[k] for k in z.files if k != "meta"}
    return meta, arrays


def state_dict(arch, fp16_values=False):
    """The seeded synthetic CLIP (fp16_values: rounded to fp16 as the released checkpoints)."""
    from fsp_amd.clip import synth
    key = (arch, fp16_values)
    if key not in _SD_CACHE:
        _SD_CACHE.clear()
        _SD_CACHE[key] = synth.make_state_dict(arch, seed=0, fp16_values=fp16_values)
    return _SD_CACHE[key]


def make_cfg(meta, prec, cocoop=False, truncate=True, shared=True):
    from fsp_amd.engine.config import get_cfg_default
    from fsp_amd.clip import synth
    a = synth.ARCHS[meta["arch"]]
    cfg = get_cfg_default()
    cfg.INPUT.SIZE = (a.image_resolution, a.image_resolution)
    cfg.NATIVE.TRUNCATE_PROMPTS = truncate
    cfg.NATIVE.SHARED_PREFIX = shared
    if cocoop:
        cfg.TRAINER.COCOOP.N_CTX = meta["n_ctx"]
        cfg.TRAINER.COCOOP.CTX_INIT = meta["ctx_init"]
        cfg.TRAINER.COCOOP.PREC = prec
        cfg.TRAINER.COCOOP.USE_FOCAL_LOSS = bool(meta["focal"])
        if meta["focal"]:
            cfg.DATASET.PER_CLASS_SHOTS = [4, 1, 2, 5, 3]
    else:
        c = cfg.TRAINER.COOP
        c.N_CTX = meta["n_ctx"] if not meta["ctx_init"] else 4
        c.CTX_INIT = meta["ctx_init"]
        c.CSC = bool(meta["csc"])
        c.CLASS_TOKEN_POSITION = meta["position"]
        c.PREC = prec
        c.LOSS_TYPE = meta["loss_type"]
        if meta["loss_type"] == "focal":
            cfg.DATASET.PER_CLASS_SHOTS = [4, 1, 2, 0, 3] if meta["arch"] == "tiny" else [16, 16, 16, 1, 1, 1]
    return cfg


def run_native(meta, arrays, prec, cocoop=False, dev="cuda", truncate=True, shared=True, fp16_values=False):
    """Returns dict with image_features, logits, loss, grads, ctx_after_step (numpy)."""
    from fsp_amd.clip import synth
    from fsp_amd.clip.model import build_model
    from fsp_amd.engine.optim import FusedSGD
    from fsp_amd.trainers import coop as C, cocoop as CC
    a = synth.ARCHS[meta["arch"]]
    cfg = make_cfg(meta, prec, cocoop, truncate, shared)
    clip = build_model(state_dict(meta["arch"], fp16_values), prec=prec, device=dev)
    names = synth.synthetic_classnames(meta["n_cls"])
    mod = CC if cocoop else C
    model = mod.CustomCLIP(cfg, names, clip)
    pl = model.prompt_learner
    out = {"split_modes": (getattr(clip.text, "split_mode", None), getattr(clip.visual, "split_mode", None)),
           "packed": pl.layout.pack is not None, "P": getattr(pl.layout, "P", 0),
           "prefix_input": pl.layout.shape(meta["batch"] if cocoop else 1).prefix_input}
    with torch.no_grad():
        if arrays.get("ctx0") is not None:
            pl.ctx.copy_(torch.from_numpy(arrays["ctx0"]).to(dev))
        if cocoop:
            mn = synth.make_meta_net(a.embed_dim, a.transformer_width, seed=4)
            for k, v in mn.items():
                dict(pl.named_parameters())[k].copy_(torch.from_numpy(v).to(dev))
    for n, p in model.named_parameters():
        if "prompt_learner" not in n:
            p.requires_grad_(False)
    out["ctx0"] = pl.ctx.detach().cpu().numpy().copy()
    B = meta["batch"]
    img = torch.from_numpy(synth.make_images(B, a.image_resolution, seed=1)).to(dev)
    img2 = torch.from_numpy(synth.make_images(B, a.image_resolution, seed=5)).to(dev)
    lbl = torch.from_numpy(synth.make_labels(B, meta["n_cls"], seed=2)).to(dev)
    if arrays.get("tokenized") is not None:
        assert (pl.tokenized_prompts.numpy() == arrays["tokenized"]).all(), "tokenization differs"
    model.eval()
    with torch.no_grad():
        out["image_features"] = model.image_encoder(img).cpu().numpy()
        if not cocoop:
            out["text_features"] = model.text_features().cpu().numpy()
            out["logits"] = model.forward_once(img).cpu().numpy()
        else:
            out["logits"] = model(img).cpu().numpy()
    model.train()
    if not cocoop and meta["loss_type"] == "simclr":
        loss = model(img, None, img2)
    else:
        loss = model(img, lbl)
    loss.backward()
    out["loss"] = float(loss.item())
    out["grad_ctx"] = pl.ctx.grad.detach().cpu().numpy()
    if cocoop:
        for k, p in pl.named_parameters():
            if k.startswith("meta_net"):
                out["grad_" + k] = p.grad.detach().cpu().numpy()
    opt = FusedSGD([p for p in pl.parameters() if p.requires_grad], lr=0.002, momentum=0.9, weight_decay=5e-4)
    opt.step()
    out["ctx_after_step"] = pl.ctx.detach().cpu().numpy()
    return out


def rel_err(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.abs(a - b).max() / (np.abs(b).max() + 1e-30))


def cos_err(a, b):
    """max over rows of 1 - cos(a_row, b_row)."""
    a = np.asarray(a, np.float64).reshape(len(a), -1)
    b = np.asarray(b, np.float64).reshape(len(b), -1)
    c = (a * b).sum(1) / np.linalg.norm(a, axis=1) / np.linalg.norm(b, axis=1)
    return float((1 - c).max())
