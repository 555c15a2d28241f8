"""Deep-prompt trainers on the GPU against the REFERENCE's own outputs
(tests/golden/make_golden_deep.py ran IVLP / MaPLe / PromptSRC on clip/model.py's prompted
blocks): logits, loss and the gradient of every trainable tensor (ctx, text deep prompts,
VPT and its deep prompts, MaPLe's projections), through the native text encoder with deep
prompts and the prompted ViT's native input-grad backward.

Gates: PREC fp32 -- |d logit| <= 1e-3, loss rel <= 1e-4, grads rel <= 1e-3 (ctx) and <= 4e-3
for the tensors the reference casts to fp16 per sequence (test_oracle_deep.grad_tol);
PREC fp16 -- |d logit| <= 0.05 at scale 100, |d loss| <= 0.05, 1 - cos(grad) <= 5e-3.
"""
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from parity_util import GOLDEN, load_fixture, rel_err, state_dict
from deep_util import init_params, grad_of

pytestmark = pytest.mark.gpu

CASES = ["ivlp_tiny4", "ivlp_tiny4_shallow", "promptsrc_tiny4", "ivlp_vitb16_c3", "maple_vitb32_c3"]


def cos_err(a, b):
    a, b = np.asarray(a, np.float64).ravel(), np.asarray(b, np.float64).ravel()
    return float(1 - a @ b / (np.linalg.norm(a) * np.linalg.norm(b) + 1e-30))


def grad_tol(name):
    return 4e-3 if ("VPT" in name or "compound" in name or "proj" in name) else 1e-3


def build(name, prec, dev):
    from fsp_amd.clip import synth
    from fsp_amd.clip.model import build_model
    from fsp_amd.engine.config import get_cfg_default
    from fsp_amd.trainers import deep as D
    meta, ref = load_fixture(name)
    a = synth.ARCHS[meta["arch"]]
    cfg = get_cfg_default()
    cfg.INPUT.SIZE = (a.image_resolution, a.image_resolution)
    names = synth.synthetic_classnames(meta["n_cls"])
    clip = build_model(state_dict(meta["arch"]), prec=prec, device=dev, vision_grad=True)
    if name.startswith("maple"):
        s = cfg.TRAINER.MAPLE
        s.N_CTX, s.CTX_INIT, s.PREC, s.PROMPT_DEPTH = meta["n_ctx"], meta["ctx_init"], prec, meta["depth"]
        model = D.MaPLeCustomCLIP(cfg, names, clip)
    else:
        sec = "PROMPTSRC" if name.startswith("promptsrc") else "IVLP"
        s = cfg.TRAINER[sec]
        s.N_CTX_TEXT, s.N_CTX_VISION, s.CTX_INIT, s.PREC = (meta["n_ctx_text"], meta["n_ctx_vision"],
                                                             meta["ctx_init"], prec)
        s.PROMPT_DEPTH_TEXT, s.PROMPT_DEPTH_VISION = meta["depth_text"], meta["depth_vision"]
        model = (D.PromptSRCCustomCLIP if sec == "PROMPTSRC" else D.IVLPCustomCLIP)(cfg, names, clip, *(
            () if sec == "PROMPTSRC" else (s,)))
    model = model.to(dev)
    params = dict(model.named_parameters())
    shapes = {k: tuple(p.shape) for k, p in params.items()}
    init = init_params(meta, ref, shapes)
    assert set(meta["trainable"]) <= set(params), set(meta["trainable"]) - set(params)
    with torch.no_grad():
        for k, v in init.items():
            params[k].copy_(torch.from_numpy(v).to(dev))
    for k, p in params.items():
        p.requires_grad_(k in meta["trainable"])
    img = torch.from_numpy(synth.make_images(meta["batch"], a.image_resolution, seed=1)).to(dev)
    lbl = torch.from_numpy(synth.make_labels(meta["batch"], meta["n_cls"], seed=2)).to(dev)
    return meta, ref, model, params, img, lbl


def run(name, prec, dev):
    meta, ref, model, params, img, lbl = build(name, prec, dev)
    model.eval()
    with torch.no_grad():
        logits = model(img).float().cpu().numpy()
    model.train()
    if name.startswith("promptsrc"):
        loss_ce, txt, fixed, zs, imf, zs_logits, lg = model(img, lbl)
        loss = loss_ce + F.l1_loss(txt, fixed) * 25 + F.l1_loss(imf, zs) * 10 + F.kl_div(
            F.log_softmax(lg, dim=1), F.log_softmax(zs_logits, dim=1), reduction="sum", log_target=True) / lg.numel()
    else:
        loss = model(img, lbl)
    loss.backward()
    grads = {k: params[k].grad.float().cpu().numpy() for k in meta["trainable"]}
    return meta, ref, logits, float(loss.detach()), grads


@pytest.mark.parametrize("prec", ["fp32", "fp16"])
@pytest.mark.parametrize("name", CASES)
def test_deep_trainer_matches_reference(dev, name, prec):
    if not os.path.exists(os.path.join(GOLDEN, name + ".npz")):
        pytest.skip("fixture not generated")
    meta, ref, logits, loss, grads = run(name, prec, dev)
    report = {"logit_abs": float(np.abs(logits - ref["logits"]).max()), "loss_abs": abs(loss - float(ref["loss"]))}
    for k, g in grads.items():
        r, rows = grad_of(ref, k)
        report[k] = rel_err(g[rows], r) if prec == "fp32" else cos_err(g[rows], r)
    print("deep", name, prec, report)
    if prec == "fp32":
        assert report["logit_abs"] <= 1e-3
        assert rel_err(loss, ref["loss"]) <= 1e-4
        for k in grads:
            assert report[k] <= grad_tol(k), (k, report[k])
    else:
        assert report["logit_abs"] <= 0.05
        assert report["loss_abs"] <= 0.05
        for k in grads:
            assert report[k] <= 5e-3, (k, report[k])


def test_prompted_vit_without_prompts_is_the_plain_vit(dev):
    """clipk_vit_forward_prompted with no prompt rows == clipk_vit_forward (same kernels up to
    the split into the shared layer loop)."""
    from fsp_amd.clip import synth
    from fsp_amd.clip.model import build_model
    for prec in ("fp32", "fp16"):
        clip = build_model(state_dict("tiny4"), prec=prec, device=dev, vision_grad=True)
        img = torch.from_numpy(synth.make_images(3, 32, seed=9)).to(dev)
        a = clip.visual(img)
        b, _ = clip.visual.forward_prompted(img, torch.zeros(0, 128, device=dev))
        tol = 1e-5 if prec == "fp32" else 2e-2
        assert float((a - b).abs().max()) <= tol * float(a.abs().max()), prec


def test_deep_text_prompts_reach_the_output(dev):
    """DeepTextEncodeFn on the packed layout: the prompts change the text features and
    receive a finite, non-zero gradient (their exact values are pinned by the fixtures)."""
    from fsp_amd.clip import synth
    from fsp_amd.clip.model import build_model, TextEncodeFn, DeepTextEncodeFn
    from fsp_amd.engine.config import get_cfg_default
    from fsp_amd.trainers.deep import VLPromptLearner
    clip = build_model(state_dict("tiny4"), prec="fp32", device=dev, vision_grad=False)
    cfg = get_cfg_default()
    cfg.INPUT.SIZE = (32, 32)
    s = cfg.TRAINER.IVLP
    s.N_CTX_TEXT, s.CTX_INIT = 4, "a photo of a"
    pl = VLPromptLearner(s, synth.synthetic_classnames(6), clip, cfg)
    x0 = pl.assemble().detach()
    shape = pl.layout.shape(1)
    plain = TextEncodeFn.apply(x0, clip.text, shape)
    assert shape.packed
    deep = torch.randn(1, 4, 128, device=dev, requires_grad=True)
    out = DeepTextEncodeFn.apply(x0.clone().requires_grad_(True), deep, clip.text, shape)
    assert float((out - plain).abs().max()) > 1e-3
    out.sum().backward()
    assert torch.isfinite(deep.grad).all() and float(deep.grad.abs().max()) > 0


def _trainer(name, outdir, dev):
    """A registry-built deep trainer on tiny4 with an in-memory data manager."""
    import contextlib
    import io
    import fsp_amd.trainers  # noqa: F401
    from fsp_amd.clip import synth
    from fsp_amd.engine.config import get_cfg_default
    from fsp_amd.engine.registry import TRAINER_REGISTRY
    cfg = get_cfg_default()
    cfg.INPUT.SIZE = (32, 32)
    cfg.MODEL.BACKBONE.NAME = "tiny4"
    cfg.OUTPUT_DIR = str(outdir)
    cfg.OPTIM.MAX_EPOCH = 2
    cfg.OPTIM.WARMUP_EPOCH = 1
    cfg.OPTIM.WARMUP_TYPE = "constant"
    cfg.TEST.NO_TEST = True
    cfg.TRAINER.NAME = name
    sec = {"IVLP": "IVLP", "MaPLe": "MAPLE", "PromptSRC": "PROMPTSRC"}[name]
    s = cfg.TRAINER[sec]
    s.PREC = "fp32"
    if sec == "MAPLE":
        s.PROMPT_DEPTH = 3
    else:
        s.PROMPT_DEPTH_TEXT = s.PROMPT_DEPTH_VISION = 3
    names = synth.synthetic_classnames(6)
    imgs = torch.from_numpy(synth.make_images(8, 32, seed=3)).to(dev)
    lbls = torch.from_numpy(synth.make_labels(8, 6, seed=4)).to(dev)

    class DM:
        class dataset:
            classnames = names
            lab2cname = {i: n for i, n in enumerate(names)}
        train_loader_x = [{"img": imgs[:4], "label": lbls[:4]}, {"img": imgs[4:], "label": lbls[4:]}]
        test_loader = [{"img": imgs, "label": lbls}]
        val_loader = None
        num_classes = 6

    with contextlib.redirect_stdout(io.StringIO()):
        return TRAINER_REGISTRY.get(name)(cfg, dm=DM())


@pytest.mark.parametrize("name", ["IVLP", "MaPLe", "PromptSRC"])
def test_deep_trainer_train_test_checkpoint(dev, tmp_path, name):
    """The registry-built trainers train (loss finite, prompts move, LR stepped at the epoch's
    last batch; PromptSRC's GPA average loaded after the last epoch), test() follows the Dassl
    contract, and the saved checkpoint (the reference's parameter names) loads back."""
    tr = _trainer(name, tmp_path / "out", dev)
    before = {k: p.detach().clone() for k, p in tr.model.named_parameters() if p.requires_grad}
    assert before and all(("prompt_learner" in k) or ("VPT" in k) for k in before)
    losses = []
    fb = tr.forward_backward
    tr.forward_backward = lambda b: losses.append(float(fb(b)["loss"])) or {"loss": losses[-1]}
    for tr.epoch in range(tr.max_epoch):
        tr.run_epoch()
        tr.after_epoch()
    assert len(losses) == 4 and all(np.isfinite(losses))
    moved = [k for k, p in tr.model.named_parameters() if k in before and not torch.equal(p.detach(), before[k])]
    assert moved, "no prompt parameter changed"
    y_true, y_pred = tr.test(return_pred=True)
    assert len(y_true) == len(y_pred) == 8
    assert isinstance(tr.test(), float)
    saved = {k: p.detach().clone() for k, p in tr.model.named_parameters()}
    tr2 = _trainer(name, tmp_path / "out2", dev)
    tr2.load_model(str(tmp_path / "out"), epoch=tr.max_epoch)
    for k, p in tr2.model.named_parameters():
        if k in before:
            assert torch.equal(p.detach(), saved[k]), k
