"""End-to-end parity of the native CoOp/CoCoOp path against golden vectors produced by
the REFERENCE itself (tests/golden/make_golden.py), through the C-ABI.

Tolerances (stated here):
* PREC "fp32" (f32-input MFMA, fp32 everything): |d logit| <= 1e-3 absolute (the
  north-star figure), features / loss / ctx-after-step rel err <= 1e-4, gradients
  rel err <= 1e-3 (prompt truncation to L_eff only reorders fp32 sums).
* PREC "fp16" (fp16 forward GEMM operands and 16-bit residual stream, fp16 backward
  operands, fp32 accumulate / LayerNorm statistics / softmax):
  1 - cos(feature) <= 5e-4, |d logit| <= 5e-4 * logit_scale (= the cosine bound at
  scale 100), |d loss| <= 0.05 (the same logit bound through a CE/focal loss, whose
  Lipschitz constant w.r.t. the max-norm of the logits is <= 2 * alpha_max here),
  gradient 1 - cos <= 2e-3.
* PREC "bf16" (bf16 forward and backward operands, bf16 residual stream): the SURVEY
  §8(c) bf16 gate 1 - cos(feature) <= 5e-3, |d logit| <= 5e-3 * 100, |d loss| <= 0.5,
  gradient 1 - cos <= 1e-2.
* PREC "amp" (fp16 forward as PREC fp16, bf16 backward operands): the fp16 forward gates,
  the bf16 gradient gate.
Every case runs twice: on the shared-prefix packed row layout (default; the prompt's
SOT + context rows encoded once per image / class set, rows past each EOT dropped) and
on the plain [B*C, L] layout (NATIVE.SHARED_PREFIX False); both against the same vectors.
Accuracy/argmax parity is not asserted: with random weights the logits are clustered
 and argmax is ill-conditioned.
"""
import os

import numpy as np
import pytest

from parity_util import load_fixture, run_native, rel_err, cos_err

pytestmark = pytest.mark.gpu

TINY_COOP = ["coop_tiny_end_csc0_ce", "coop_tiny_end_csc1_ce", "coop_tiny_middle_csc0_ce",
             "coop_tiny_middle_csc1_ce", "coop_tiny_front_csc0_ce", "coop_tiny_front_csc1_ce",
             "coop_tiny_end_focal", "coop_tiny_end_simclr", "coop_tiny_ctxinit_ce", "coop_tinyp8_end_ce"]
TINY_COCOOP = ["cocoop_tiny_ctxinit_ce", "cocoop_tiny_focal"]
FULL_COOP = ["coop_vitb32_c10", "coop_vitb16_c6_focal", "coop_vitl14_c4"]
FULL_COCOOP = ["cocoop_vitb16_c4", "cocoop_vitl14_336_c3"]


PRECS = ["fp32", "fp32s", "fp16", "bf16", "amp"]
FP32_CLASS = ("fp32", "fp32s")  # held to the fp32 gates (north-star |d logit| <= 1e-3)
# 16-bit gates: (feature 1-cos [logit bound = it x 100], |d loss|, gradient 1-cos)
TOL16 = {"fp16": (5e-4, 0.05, 2e-3), "bf16": (5e-3, 0.5, 1e-2), "amp": (5e-4, 0.05, 1e-2)}

SHOULD_PACK = {"coop_tiny_end_csc0_ce", "coop_tiny_middle_csc0_ce", "coop_tiny_end_focal", "coop_tiny_end_simclr",
               "coop_tiny_ctxinit_ce", "coop_tinyp8_end_ce", "cocoop_tiny_ctxinit_ce", "cocoop_tiny_focal",
               "coop_vitb32_c10", "coop_vitb16_c6_focal", "coop_vitl14_c4", "cocoop_vitb16_c4",
               "cocoop_vitl14_336_c3"}


def _check(name, cocoop, prec, dev, layout="packed", split_modes=None):
    meta, ref = load_fixture(name)
    out = run_native(meta, ref, prec, cocoop=cocoop, dev=str(dev), shared=layout == "packed",
                     fp16_values=bool(meta.get("fp16_values", False)))
    if split_modes is not None:
        assert out["split_modes"] == split_modes, out["split_modes"]
    assert out["packed"] == (layout == "packed" and name in SHOULD_PACK), (name, layout, out["packed"])
    grads = [k for k in ref if k.startswith("grad_")]
    report = {}
    if prec in FP32_CLASS:
        report["logit_abs"] = float(np.abs(out["logits"] - ref["logits"]).max())
        report["imf"] = rel_err(out["image_features"], ref["image_features"])
        report["loss"] = rel_err(out["loss"], ref["loss"])
        report["step"] = rel_err(out["ctx_after_step"], ref["ctx_after_step"])
        for g in grads:
            report[g] = rel_err(out[g], ref[g])
        print(name, prec, report)
        assert report["logit_abs"] <= 1e-3
        assert report["imf"] <= 1e-4
        assert report["loss"] <= 1e-4
        assert report["step"] <= 1e-4
        for g in grads:
            assert report[g] <= 1e-3, (g, report[g])
        if "text_features" in ref:
            assert rel_err(out["text_features"], ref["text_features"]) <= 1e-4
    else:
        fwd_cos, loss_tol, grad_cos = TOL16[prec]
        report["imf_cos"] = cos_err(out["image_features"], ref["image_features"])
        report["logit_abs"] = float(np.abs(out["logits"] - ref["logits"]).max())
        report["loss_abs"] = abs(out["loss"] - float(ref["loss"]))
        for g in grads:
            report[g] = cos_err(out[g].reshape(1, -1), ref[g].reshape(1, -1))
        if "text_features" in ref:
            report["txt_cos"] = cos_err(out["text_features"], ref["text_features"])
        print(name, prec, layout, report)
        assert report["imf_cos"] <= fwd_cos
        assert report["logit_abs"] <= fwd_cos * 100.0
        assert report["loss_abs"] <= loss_tol
        for g in grads:
            assert report[g] <= grad_cos, (g, report[g])
        if "text_features" in ref:
            assert report["txt_cos"] <= fwd_cos


@pytest.mark.parametrize("layout", ["packed", "plain"])
@pytest.mark.parametrize("prec", PRECS)
@pytest.mark.parametrize("name", TINY_COOP)
def test_coop_tiny(dev, name, prec, layout):
    _check(name, False, prec, dev, layout)


@pytest.mark.parametrize("layout", ["packed", "plain"])
@pytest.mark.parametrize("prec", PRECS)
@pytest.mark.parametrize("name", TINY_COCOOP)
def test_cocoop_tiny(dev, name, prec, layout):
    _check(name, True, prec, dev, layout)


@pytest.mark.parametrize("layout", ["packed", "plain"])
@pytest.mark.parametrize("prec", PRECS)
@pytest.mark.parametrize("name", FULL_COOP)
def test_coop_full(dev, name, prec, layout):
    _check(name, False, prec, dev, layout)


@pytest.mark.parametrize("layout", ["packed", "plain"])
@pytest.mark.parametrize("prec", PRECS)
@pytest.mark.parametrize("name", FULL_COCOOP)
def test_cocoop_full(dev, name, prec, layout):
    _check(name, True, prec, dev, layout)


_ORACLE_CACHE = {}


def _cocoop_oracle(arch, n_cls, batch, seed_img=1, fp16_values=False):
    """CPU oracle (pinned by the golden vectors) for a CoCoOp configuration too large for
    a committed fixture ("a photo of a" context, CE): logits, loss, d ctx, d meta_net.
    Cached per configuration (the ViT-B/16 C = 1000 case costs ~5 TFLOP on the host)."""
    key = (arch, n_cls, batch, seed_img, fp16_values)
    if key in _ORACLE_CACHE:
        return _ORACLE_CACHE[key]
    import torch
    from oracle import clip_oracle as O
    from fsp_amd.clip import synth
    from fsp_amd.clip.tokenizer import tokenize
    a = synth.ARCHS[arch]
    p = O.as_torch_sd(synth.make_state_dict(arch, seed=0, fp16_values=fp16_values))
    mp = {k: torch.from_numpy(v).requires_grad_(True)
          for k, v in synth.make_meta_net(a.embed_dim, a.transformer_width, seed=4).items()}
    names = synth.synthetic_classnames(n_cls)
    tok = torch.from_numpy(tokenize(["a photo of a " + n + "." for n in names]).astype(np.int64))
    emb = O.token_embed(p, tok)
    ctx = emb[0, 1:5].clone().requires_grad_(True)
    img = torch.from_numpy(synth.make_images(batch, a.image_resolution, seed=seed_img))
    L = int(tok.argmax(-1).max()) + 1
    logits = O.cocoop_logits(p, mp, img, ctx, emb[:, :1], emb[:, 5:], tok, L)
    y = torch.from_numpy(synth.make_labels(batch, n_cls, seed=2))
    loss = torch.nn.functional.cross_entropy(logits, y)
    loss.backward()
    out = {"logits": logits.detach().numpy(), "loss": float(loss.detach()), "grad_ctx": ctx.grad.numpy(),
           "ctx0": ctx.detach().numpy()}
    for k, v in mp.items():
        out["grad_" + k] = v.grad.numpy()
    _ORACLE_CACHE.clear()
    _ORACLE_CACHE[key] = out
    return out


@pytest.mark.parametrize("prec", ["fp32", "fp32s", "fp16"])
@pytest.mark.parametrize("layout", ["packed", "plain"])
def test_cocoop_large_rows_vs_oracle(dev, prec, layout):
    """tiny CLIP, C = 2000 classes x B = 3 images: 66k text rows, so the large-M GEMM
    paths (persistent 256x256) run inside the full model; checked against the oracle."""
    meta = {"arch": "tiny", "n_cls": 2000, "batch": 3, "n_ctx": 4, "ctx_init": "a photo of a", "focal": 0}
    ref = _cocoop_oracle("tiny", 2000, 3)
    out = run_native(meta, {"ctx0": ref["ctx0"], "tokenized": None}, prec, cocoop=True, dev=str(dev),
                     shared=layout == "packed")
    assert out["packed"] == (layout == "packed")
    if prec in FP32_CLASS:
        assert float(np.abs(out["logits"] - ref["logits"]).max()) <= 1e-3
        assert rel_err(out["grad_ctx"], ref["grad_ctx"]) <= 1e-3
    else:
        assert float(np.abs(out["logits"] - ref["logits"]).max()) <= 5e-2
        assert cos_err(out["grad_ctx"].reshape(1, -1), ref["grad_ctx"].reshape(1, -1)) <= 2e-3


@pytest.mark.parametrize("prec", ["fp32", "fp32s", "fp16", "bf16", "amp"])
def test_headline_shape_vs_oracle(dev, prec):
    """The benchmark workload's shape (BASELINE config 3: CoCoOp ViT-B/16, C = 1000 classes,
    n_ctx 4 "a photo of a", shared-prefix packed rows, the 192/256-row GEMM tiles and the
    W = 512 prefix-attention tiling) at B = 2 images, against the CPU oracle: logits, CE loss,
    d ctx and d meta_net. Gates as _check (fp32: |d logit| <= 1e-3, grads rel <= 1e-3)."""
    meta = {"arch": "ViT-B/16", "n_cls": 1000, "batch": 2, "n_ctx": 4, "ctx_init": "a photo of a", "focal": 0}
    ref = _cocoop_oracle("ViT-B/16", 1000, 2)
    out = run_native(meta, {"ctx0": None, "tokenized": None}, prec, cocoop=True, dev=str(dev))
    assert out["packed"]
    np.testing.assert_array_equal(out["ctx0"], ref["ctx0"])
    grads = [k for k in ref if k.startswith("grad_")]
    report = {"logit_abs": float(np.abs(out["logits"] - ref["logits"]).max()),
              "loss_abs": abs(out["loss"] - ref["loss"])}
    if prec in FP32_CLASS:
        report.update({g: rel_err(out[g], ref[g]) for g in grads})
        print("headline", prec, report)
        assert report["logit_abs"] <= 1e-3
        assert report["loss_abs"] <= 1e-4 * max(1.0, abs(ref["loss"]))
        for g in grads:
            assert report[g] <= 1e-3, (g, report[g])
    else:
        fwd_cos, loss_tol, grad_cos = TOL16[prec]
        report.update({g: cos_err(out[g].reshape(1, -1), ref[g].reshape(1, -1)) for g in grads})
        print("headline", prec, report)
        assert report["logit_abs"] <= fwd_cos * 100.0
        assert report["loss_abs"] <= loss_tol
        for g in grads:
            assert report[g] <= grad_cos, (g, report[g])


@pytest.mark.parametrize("prec", ["fp32", "fp16"])
@pytest.mark.parametrize("ensemble", [False, True])
def test_zeroshot_clip_vs_oracle(dev, prec, ensemble):
    """ZeroshotCLIP / ZeroshotCLIP2 (zsclip.py:32-99) through the registry, vs the CPU oracle
    (encode_image / encode_text pinned by the golden vectors): logits = exp(logit_scale) *
    cos(image, class prompt feature); ZeroshotCLIP2 averages normalised template features.
    Templates limited to ones the fallback tokenizer covers (no BPE vocab on the GPU box)."""
    import torch
    from oracle import clip_oracle as O
    from fsp_amd.clip import synth
    from fsp_amd.clip.tokenizer import tokenize
    from fsp_amd.engine.config import get_cfg_default
    from fsp_amd.engine.registry import TRAINER_REGISTRY
    from fsp_amd.data.synthetic import SyntheticDataManager
    from fsp_amd.trainers import zsclip
    arch, n_cls, B = "ViT-B/32", 12, 3
    a = synth.ARCHS[arch]
    cfg = get_cfg_default()
    cfg.MODEL.BACKBONE.NAME = arch
    cfg.INPUT.SIZE = (a.image_resolution, a.image_resolution)
    cfg.DATASET.NAME = "ImageNet"
    cfg.TRAINER.COOP.PREC = prec
    cfg.TRAINER.NAME = "ZeroshotCLIP2" if ensemble else "ZeroshotCLIP"
    dm = SyntheticDataManager(n_cls, a.image_resolution, B, n_batches=1, device=str(dev))
    cls = TRAINER_REGISTRY.get(cfg.TRAINER.NAME)
    templates = ["a photo of a {}.", "X X X X {}."] if ensemble else ["a photo of a {}."]
    if ensemble:
        cls = type("ZS2Probe", (cls,), {"templates": templates})
    tr = cls(cfg, dm=dm)
    img = torch.from_numpy(synth.make_images(B, a.image_resolution, seed=1)).to(dev)
    with torch.no_grad():
        logits = tr.model_inference(img).cpu().numpy()
    p = O.as_torch_sd(synth.make_state_dict(arch, seed=0))
    names = synth.synthetic_classnames(n_cls)
    feats = 0
    for t in templates:
        tok = torch.from_numpy(tokenize([t.format(n) for n in names]).astype(np.int64))
        with torch.no_grad():
            f = O.encode_text(p, O.token_embed(p, tok), tok)
        feats = feats + O.normalize(f)
    feats = O.normalize(feats / len(templates))
    with torch.no_grad():
        imf = O.normalize(O.encode_image(p, torch.from_numpy(synth.make_images(B, a.image_resolution, seed=1))))
    ref = (float(np.exp(float(p["logit_scale"]))) * imf @ feats.t()).numpy()
    tol = 1e-3 if prec == "fp32" else 5e-4 * 100.0
    assert float(np.abs(logits - ref).max()) <= tol


@pytest.mark.parametrize("prec", ["fp32", "fp16"])
@pytest.mark.parametrize("name,cocoop", [("cocoop_tiny_ctxinit_ce", True), ("cocoop_vitb16_c4", True),
                                         ("coop_tiny_end_csc0_ce", False), ("coop_tiny_middle_csc0_ce", False)])
def test_prefix_input_mode_is_exact(dev, name, prec, cocoop, monkeypatch):
    """clipk_encoder_set_input_rows(1) (layer 0's LN1 / qkv on the class rows once, copied to every
    group; dx0 formed on the prefix rows only) against mode 0 on the same packed layout: the
    same per-row arithmetic, so logits, loss and every prompt gradient agree to fp32 rounding
    (1e-6 relative; 16-bit: 1e-3). cocoop_tiny has 3 images (groups 1 and 2 take the copy and
    the compact-row scatter); the middle position keeps context slots among the class rows, so
    it must stay in mode 0."""
    from fsp_amd.trainers import prompt_base
    meta, ref = load_fixture(name)
    outs = {}
    for mode in (False, True):
        monkeypatch.setattr(prompt_base, "PREFIX_INPUT", mode)
        outs[mode] = run_native(meta, ref, prec, cocoop=cocoop, dev=str(dev))
        assert outs[mode]["packed"]
    tol = 1e-6 if prec == "fp32" else 1e-3
    for k in ["logits", "loss", "ctx_after_step"] + [k for k in outs[True] if k.startswith("grad_")]:
        assert rel_err(outs[True][k], outs[False][k]) <= tol, (k, rel_err(outs[True][k], outs[False][k]))
    if "middle" in name:
        assert not _layout_prefix_input(meta, prec, cocoop, dev)
    else:
        assert _layout_prefix_input(meta, prec, cocoop, dev)


def _layout_prefix_input(meta, prec, cocoop, dev):
    from parity_util import make_cfg, state_dict
    from fsp_amd.clip import synth
    from fsp_amd.clip.model import build_model
    from fsp_amd.trainers import coop as C, cocoop as CC
    cfg = make_cfg(meta, prec, cocoop)
    clip = build_model(state_dict(meta["arch"]), prec=prec, device=str(dev))
    model = (CC if cocoop else C).CustomCLIP(cfg, synth.synthetic_classnames(meta["n_cls"]), clip)
    return model.prompt_learner.layout.shape(2).prefix_input


def _coop_oracle(arch, n_cls, batch, n_ctx=16, seed_ctx=11):
    """CPU oracle for CoOp (class token "end", shared random context, CE) at a size too large
    for a committed fixture: logits, loss, d ctx. Prompts truncated to L_eff (exact, SURVEY
    §8 a6, pinned by test_oracle_golden). Cached per configuration."""
    key = ("coop", arch, n_cls, batch, n_ctx, seed_ctx)
    if key in _ORACLE_CACHE:
        return _ORACLE_CACHE[key]
    import torch
    from oracle import clip_oracle as O
    from fsp_amd.clip import synth
    from fsp_amd.clip.tokenizer import tokenize
    a = synth.ARCHS[arch]
    p = O.as_torch_sd(synth.make_state_dict(arch, seed=0))
    names = synth.synthetic_classnames(n_cls)
    tok = torch.from_numpy(tokenize([" ".join(["X"] * n_ctx) + " " + n + "." for n in names]).astype(np.int64))
    emb = O.token_embed(p, tok)
    ctx0 = (np.random.RandomState(seed_ctx).standard_normal((n_ctx, a.transformer_width)) * 0.02).astype(np.float32)
    ctx = torch.from_numpy(ctx0.copy()).requires_grad_(True)
    img = torch.from_numpy(synth.make_images(batch, a.image_resolution, seed=1))
    L = int(tok.argmax(-1).max()) + 1
    logits = O.coop_logits(p, img, ctx, emb[:, :1], emb[:, 1 + n_ctx:], tok, [0] * n_cls, "end", L)
    y = torch.from_numpy(synth.make_labels(batch, n_cls, seed=2))
    loss = torch.nn.functional.cross_entropy(logits, y)
    loss.backward()
    out = {"logits": logits.detach().numpy(), "loss": float(loss.detach()), "grad_ctx": ctx.grad.numpy(),
           "ctx0": ctx0, "L": L}
    _ORACLE_CACHE.clear()
    _ORACLE_CACHE[key] = out
    return out


def _gate(ref, out, prec, tag):
    grads = [k for k in ref if k.startswith("grad_")]
    report = {"logit_abs": float(np.abs(out["logits"] - ref["logits"]).max()),
              "loss_abs": abs(out["loss"] - ref["loss"])}
    if prec in FP32_CLASS:
        report.update({g: rel_err(out[g], ref[g]) for g in grads})
        print(tag, prec, report)
        assert report["logit_abs"] <= 1e-3
        assert report["loss_abs"] <= 1e-4 * max(1.0, abs(ref["loss"]))
        for g in grads:
            assert report[g] <= 1e-3, (g, report[g])
    else:
        fwd_cos, loss_tol, grad_cos = TOL16[prec]
        report.update({g: cos_err(out[g].reshape(1, -1), ref[g].reshape(1, -1)) for g in grads})
        print(tag, prec, report)
        assert report["logit_abs"] <= fwd_cos * 100.0
        assert report["loss_abs"] <= loss_tol
        for g in grads:
            assert report[g] <= grad_cos, (g, report[g])


@pytest.mark.parametrize("prec", ["fp32", "fp32s", "fp16"])
def test_config2_coop_vitb16_c1000_vs_oracle(dev, prec):
    """BASELINE config 2 at its shape: CoOp n_ctx 16 (random shared context, class token at
    the end), ViT-B/16, C = 1000 classes, B = 2 images, CE; the shared-prefix packed layout
    with its prefix capped at P = 16 rows (SOT + 15 context slots), so the 16th context slot
    is a per-class row (prompt_base.shared_prefix_tables max_prefix) and layer 0 runs the full
    input (no prefix-input mode). Logits, loss and d ctx vs the CPU oracle."""
    meta = {"arch": "ViT-B/16", "n_cls": 1000, "batch": 2, "n_ctx": 16, "ctx_init": "", "csc": 0,
            "position": "end", "loss_type": "ce", "focal": 0}
    ref = _coop_oracle("ViT-B/16", 1000, 2, 16)
    out = run_native(meta, {"ctx0": ref["ctx0"], "tokenized": None}, prec, cocoop=False, dev=str(dev))
    assert out["packed"] and out["P"] == 16 and not out["prefix_input"]
    _gate(ref, out, prec, "config2")


@pytest.mark.parametrize("prec", ["fp32", "fp32s", "bf16"])
def test_config4_coop_vitl14_c1000_vs_oracle(dev, prec):
    """BASELINE config 4 at its full size (CoOp n_ctx 16 random shared context, class token at
    the end, ViT-L/14, bf16; PromptSRC/trainers/coop.py:351-363): C = 1,000 classes, B = 2
    images, so the W = 768 text runs its full-size GEMM tiles (the persistent 192/256-row
    tiles on N = 768 / 2,304 / 3,072) and the packed P = 16 prefix attention, vs the CPU
    oracle: logits, loss, d ctx."""
    meta = {"arch": "ViT-L/14", "n_cls": 1000, "batch": 2, "n_ctx": 16, "ctx_init": "", "csc": 0,
            "position": "end", "loss_type": "ce", "focal": 0}
    ref = _coop_oracle("ViT-L/14", 1000, 2, 16)
    out = run_native(meta, {"ctx0": ref["ctx0"], "tokenized": None}, prec, cocoop=False, dev=str(dev))
    assert out["packed"] and out["P"] == 16
    _gate(ref, out, prec, "config4")


@pytest.mark.parametrize("prec", ["fp32", "fp32s", "bf16"])
def test_config4_class_shard_slice(dev, prec):
    """Config 4's class sharding (125 classes each): the text features a
    rank encodes for its slice [lo, hi) equal rows lo..hi-1 of the full 1,000-class encoding
    (the row-wise text encoder on a different packed row count, so other GEMM grids and
    attention tiles)."""
    import torch
    from parity_util import make_cfg, state_dict
    from fsp_amd.clip import synth
    from fsp_amd.clip.model import build_model
    from fsp_amd.trainers import coop as C
    meta = {"arch": "ViT-L/14", "n_cls": 1000, "batch": 2, "n_ctx": 16, "ctx_init": "", "csc": 0,
            "position": "end", "loss_type": "ce", "focal": 0}
    cfg = make_cfg(meta, prec)
    clip = build_model(state_dict(meta["arch"]), prec=prec, device=str(dev))
    names = synth.synthetic_classnames(1000)
    ctx0 = torch.from_numpy((np.random.RandomState(11).standard_normal((16, 768)) * 0.02).astype(np.float32))
    full = C.CustomCLIP(cfg, names, clip)
    with torch.no_grad():
        full.prompt_learner.ctx.copy_(ctx0.to(dev))
        txt_full = full.text_features().float().cpu().numpy()
    for r in (0, 3, 7):
        lo, hi = r * 125, (r + 1) * 125
        pl = C.PromptLearner(cfg, names, clip, class_range=(lo, hi))
        with torch.no_grad():
            pl.ctx.copy_(ctx0.to(dev))
            txt = C.TextEncodeFn.apply(pl.assemble(), clip.text, pl.layout.shape(1)).float().cpu().numpy()
        assert txt.shape == (125, txt_full.shape[1])
        err = rel_err(txt, txt_full[lo:hi])
        print("class shard", prec, r, err)
        assert err <= (1e-5 if prec in FP32_CLASS else 1e-2), (r, err)


@pytest.mark.parametrize("prec", ["fp32", "fp32s", "bf16"])
def test_config5_cocoop_vitl14_336_c1000_vs_oracle(dev, prec):
    """BASELINE config 5 at its full size (CoCoOp ViT-L/14@336px, bf16, "a photo of a";
    PromptSRC/trainers/cocoop.py:235-260): C = 1,000 classes, B = 2 images (577-token ViT,
    W = 768 text at its full-size GEMM tiles, packed P = 5 prefix + prefix-input mode), vs the
    CPU oracle: logits, loss, d ctx, d Meta-Net."""
    meta = {"arch": "ViT-L/14@336px", "n_cls": 1000, "batch": 2, "n_ctx": 4, "ctx_init": "a photo of a", "focal": 0}
    ref = _cocoop_oracle("ViT-L/14@336px", 1000, 2)
    out = run_native(meta, {"ctx0": None, "tokenized": None}, prec, cocoop=True, dev=str(dev))
    assert out["packed"] and out["P"] == 5 and out["prefix_input"]
    np.testing.assert_array_equal(out["ctx0"], ref["ctx0"])
    _gate(ref, out, prec, "config5")


HEADLINE = "cocoop_vitb16_c1000_b8"


@pytest.mark.parametrize("prec", ["fp32", "fp32s", "fp16"])
def test_headline_batch8_vs_golden(dev, prec):
    """The benchmark step itself -- CoCoOp ViT-B/16, C = 1,000 classes, B = 8 images, n_ctx 4
    "a photo of a", CE (47,160 packed text rows: the grid the timed N = 512 GEMMs run on) --
    against the REFERENCE's own outputs at that size (tests/golden/make_golden.py --only
    headline: logits, loss, d ctx, d Meta-Net, ctx after the SGD step), at the gates of _check
    (fp32 / fp32s |d logit| <= 1e-3, gradients rel <= 1e-3; fp16 the 16-bit gates)."""
    if not os.path.exists(os.path.join(os.path.dirname(__file__), "golden", HEADLINE + ".npz")):
        pytest.fail(f"fixture {HEADLINE}.npz missing (tests/golden/make_golden.py --only headline)")
    SHOULD_PACK.add(HEADLINE)
    _check(HEADLINE, True, prec, dev)


def test_fp32s_gradient_overflow_is_detected_and_rerun(dev, monkeypatch):
    """PREC fp32s runs the text backward on s * dtxt (s from max |dtxt|); a gradient that grows past
    fp16's 65504 inside the split-fp16 GEMM operands gives inf / NaN. The encoder flags non-finite
    returned gradients (clipk_encoder_set_status) and the Python core re-runs the backward once at
    a lower scale target. Forced here with a scale target of 2^20 (the first split of s * dtxt
    overflows): the run still meets the fp32 gates against the reference, through one re-run."""
    from fsp_amd.clip.model import TextEncoderCore
    monkeypatch.setattr(TextEncoderCore, "SPLIT_TARGET", 20)
    before = TextEncoderCore.split_retries
    _check("cocoop_vitb16_c4", True, "fp32s", dev)
    assert TextEncoderCore.split_retries == before + 1


def test_fp32s_default_target_needs_no_rerun(dev):
    from fsp_amd.clip.model import TextEncoderCore
    before = TextEncoderCore.split_retries
    _check("cocoop_vitb16_c4", True, "fp32s", dev)
    assert TextEncoderCore.split_retries == before


HEADLINE_W16 = "cocoop_vitb16_c1000_b8_w16"


@pytest.mark.parametrize("prec", ["fp32s", "fp16"])
def test_headline_batch8_w16_vs_golden(dev, prec):
    """The benched configuration exactly: CoCoOp ViT-B/16, C = 1,000, B = 8,
    n_ctx 4 "a photo of a", on fp16-VALUED weights (as the released checkpoints load and as
    bench.py's synthetic weights are made) against the reference's own outputs for those weights
    (tests/golden/make_golden.py --only headline_w16). PREC fp32s runs split mode 2 on it -- every
    GEMM CLIPK_F32S16 on the compact weights, the gamma-on-A fold, the pre-split MLP hand-offs --
    and is held to the fp32 gates; fp16 to the 16-bit gates."""
    if not os.path.exists(os.path.join(os.path.dirname(__file__), "golden", HEADLINE_W16 + ".npz")):
        pytest.fail(f"fixture {HEADLINE_W16}.npz missing (tests/golden/make_golden.py --only headline_w16)")
    SHOULD_PACK.add(HEADLINE_W16)
    _check(HEADLINE_W16, True, prec, dev, split_modes=(2, 2) if prec == "fp32s" else None)
