"""Generate golden vectors by running the REFERENCE hot path itself (CPU, fp32).

Run in the survey/build container only (needs /root/reference):
    python tests/golden/make_golden.py [--full]

The reference is imported with minimal stand-ins for modules the image lacks
(``ftfy``: identity, exact for ASCII class names; ``torchvision``: inert
transform classes, only referenced at import time; ``dassl.engine``: the real
``dassl.utils.Registry`` + ``TrainerX = object`` because the real engine imports
tensorboard). Weights/inputs come from ``fsp_amd.clip.synth`` (seeded numpy), so
only seeds, a weight digest and the reference OUTPUTS are stored in the fixtures.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference/PromptSRC"
DASSL = "/root/reference/Dassl.pytorch"
sys.path.insert(0, REPO)

from fsp_amd.clip import synth  # noqa: E402


def _install_stubs():
    ftfy = types.ModuleType("ftfy")
    ftfy.fix_text = lambda s: s
    sys.modules["ftfy"] = ftfy

    tv = types.ModuleType("torchvision")
    tr = types.ModuleType("torchvision.transforms")

    class _T:
        def __init__(self, *a, **k):
            pass

        def __call__(self, x):
            return x

    for n in ["Compose", "Resize", "CenterCrop", "ToTensor", "Normalize", "RandomResizedCrop",
              "RandomHorizontalFlip", "RandomApply", "ColorJitter", "RandomGrayscale"]:
        setattr(tr, n, _T)

    class InterpolationMode:
        BICUBIC = 3

    tr.InterpolationMode = InterpolationMode
    tv.transforms = tr
    sys.modules["torchvision"] = tv
    sys.modules["torchvision.transforms"] = tr

    sys.path.insert(0, DASSL)
    sys.path.insert(0, REF)
    import dassl  # noqa: F401  (package __init__ is import-free)
    from dassl.utils import Registry
    eng = types.ModuleType("dassl.engine")
    eng.TRAINER_REGISTRY = Registry("TRAINER")
    eng.TrainerX = object
    sys.modules["dassl.engine"] = eng


class Cfg(dict):
    """Attribute dict with .get, standing in for a yacs CfgNode."""

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e

    def __setattr__(self, k, v):
        self[k] = v


def make_cfg(size, coop=None, cocoop=None, per_class=None):
    return Cfg(
        INPUT=Cfg(SIZE=(size, size)),
        DATASET=Cfg(PER_CLASS_SHOTS=per_class),
        TRAINER=Cfg(COOP=Cfg(**(coop or {})), COCOOP=Cfg(**(cocoop or {}))),
    )


DESIGN = {"vision_depth": 0, "language_depth": 0, "vision_ctx": 0, "language_ctx": 0}


def build_clip(arch, fp16_values=False):
    """The seeded synthetic CLIP (fp16_values: every weight rounded to fp16, as the released
    checkpoints the reference loads from its fp16 archive, PromptSRC/clip/clip.py:154-180)."""
    sd = synth.make_state_dict(arch, seed=0, fp16_values=fp16_values)
    digest = synth.state_dict_digest(sd)
    tsd = {k: torch.from_numpy(v.copy()) for k, v in sd.items()}
    return tsd, digest


def sgd_after_step(module, lr=0.002):
    opt = torch.optim.SGD([p for p in module.parameters() if p.requires_grad], lr=lr,
                          momentum=0.9, weight_decay=5e-4, dampening=0, nesterov=False)
    opt.step()
    return opt


def run_coop(arch, n_cls, batch, n_ctx, position, csc, loss_type, ctx_init="", per_class=None,
             L_trunc=None):
    from clip.model import build_model
    import trainers.coop as coop
    tsd, digest = build_clip(arch)
    a = synth.ARCHS[arch]
    design = dict(DESIGN, trainer="CoOp")
    model = build_model(dict(tsd), design).float()
    cfg = make_cfg(a.image_resolution,
                   coop=dict(N_CTX=n_ctx, CTX_INIT=ctx_init, CSC=csc, CLASS_TOKEN_POSITION=position,
                             PREC="fp32", LOSS_TYPE=loss_type),
                   per_class=per_class)
    names = synth.synthetic_classnames(n_cls)
    cc = coop.CustomCLIP(cfg, names, model)
    for n, p in cc.named_parameters():
        if "prompt_learner" not in n:
            p.requires_grad_(False)
    if not ctx_init:
        ctx = synth.make_ctx(n_ctx, a.transformer_width, n_cls if csc else None, seed=3)
        with torch.no_grad():
            cc.prompt_learner.ctx.copy_(torch.from_numpy(ctx))
    ctx0 = cc.prompt_learner.ctx.detach().clone().numpy()
    img = torch.from_numpy(synth.make_images(batch, a.image_resolution, seed=1))
    img2 = torch.from_numpy(synth.make_images(batch, a.image_resolution, seed=5))
    lbl = torch.from_numpy(synth.make_labels(batch, n_cls, seed=2))
    out = dict(arch=arch, digest=digest, n_cls=n_cls, batch=batch, n_ctx=n_ctx,
               position=position, csc=int(csc), loss_type=loss_type, ctx_init=ctx_init)
    cc.eval()
    with torch.no_grad():
        imf = cc.image_encoder(img)
        prompts = cc.prompt_learner()
        txt = cc.text_encoder(prompts, cc.tokenized_prompts)
        # simclr-mode CustomCLIP.forward needs img2 even in eval (coop.py:370-377)
        logits = cc.forward_once(img) if loss_type == "simclr" else cc(img)
    cc.train()
    if loss_type == "simclr":
        loss = cc(img, None, img2)
    else:
        loss = cc(img, lbl)
    loss.backward()
    grad = cc.prompt_learner.ctx.grad.detach().clone().numpy()
    sgd_after_step(cc.prompt_learner)
    arrays = dict(ctx0=ctx0, image_features=imf.numpy(), text_features=txt.numpy(),
                  logits=logits.numpy(), loss=np.asarray(loss.item(), np.float32),
                  grad_ctx=grad, ctx_after_step=cc.prompt_learner.ctx.detach().numpy(),
                  tokenized=cc.tokenized_prompts.numpy().astype(np.int32),
                  name_lens=np.asarray(cc.prompt_learner.name_lens, np.int32))
    return out, arrays


def run_cocoop(arch, n_cls, batch, ctx_init, n_ctx, focal, per_class=None):
    from clip.model import build_model
    import trainers.cocoop as cocoop
    tsd, digest = build_clip(arch)
    a = synth.ARCHS[arch]
    design = dict(DESIGN, trainer="CoCoOp")
    model = build_model(dict(tsd), design).float()
    cfg = make_cfg(a.image_resolution,
                   cocoop=dict(N_CTX=n_ctx, CTX_INIT=ctx_init, PREC="fp32", USE_FOCAL_LOSS=focal),
                   per_class=per_class)
    names = synth.synthetic_classnames(n_cls)
    cc = cocoop.CustomCLIP(cfg, names, model)
    for n, p in cc.named_parameters():
        if "prompt_learner" not in n:
            p.requires_grad_(False)
    pl = cc.prompt_learner
    mn = synth.make_meta_net(a.embed_dim, a.transformer_width, seed=4)
    with torch.no_grad():
        if not ctx_init:
            pl.ctx.copy_(torch.from_numpy(synth.make_ctx(n_ctx, a.transformer_width, seed=3)))
        for k, v in mn.items():
            dict(pl.named_parameters())[k].copy_(torch.from_numpy(v))
    ctx0 = pl.ctx.detach().clone().numpy()
    img = torch.from_numpy(synth.make_images(batch, a.image_resolution, seed=1))
    lbl = torch.from_numpy(synth.make_labels(batch, n_cls, seed=2))
    out = dict(arch=arch, digest=digest, n_cls=n_cls, batch=batch, n_ctx=pl.n_ctx,
               ctx_init=ctx_init, focal=int(focal))
    cc.eval()
    with torch.no_grad():
        imf = cc.image_encoder(img)
        logits = cc(img)
    cc.train()
    loss = cc(img, lbl)
    loss.backward()
    grads = {"grad_ctx": pl.ctx.grad.detach().clone().numpy()}
    for k, p in pl.named_parameters():
        if k.startswith("meta_net"):
            grads["grad_" + k] = p.grad.detach().clone().numpy()
    sgd_after_step(pl)
    arrays = dict(ctx0=ctx0, image_features=imf.numpy(), logits=logits.numpy(),
                  loss=np.asarray(loss.item(), np.float32), ctx_after_step=pl.ctx.detach().numpy(),
                  tokenized=cc.tokenized_prompts.numpy().astype(np.int32), **grads)
    return out, arrays


def lr_sequences():
    """Dassl warmup+cosine LR per epoch (lr_scheduler.py), with a shim for torch 2.10
    (the reference passes ``verbose`` positionally to _LRScheduler.__init__)."""
    from dassl.optim import lr_scheduler as ls
    base = torch.optim.lr_scheduler.LRScheduler.__init__

    def init(self, optimizer, last_epoch=-1, verbose=False):
        base(self, optimizer, last_epoch)

    ls._LRScheduler.__init__ = init
    res = {}
    for max_epoch in (10, 50):
        p = torch.nn.Parameter(torch.zeros(1))
        opt = torch.optim.SGD([p], lr=0.002, momentum=0.9)
        cos = torch.optim.lr_scheduler.CosineAnnealingLR(opt, float(max_epoch))
        sch = ls.ConstantWarmupScheduler(opt, cos, 1, 1e-5)
        seq = []
        for _ in range(max_epoch):
            seq.append(opt.param_groups[0]["lr"])
            sch.step()
        res[max_epoch] = np.asarray(seq, np.float64)
    return res


def tokenizer_table():
    """Word -> ids for the synthetic prompt vocabulary (fallback when no BPE vocab)."""
    from clip.simple_tokenizer import SimpleTokenizer
    tok = SimpleTokenizer()
    words = ["x", "a", "photo", "of", "class", "."] + [str(d) for d in range(10)]
    table = {w: tok.encode(w) for w in words}
    probes = ["X X X X class7.", "a photo of a class123.", "a photo of a dog.",
              "Hello, World! it's 2 o'clock", "X " * 16 + "class999."]
    probes += template_probes()
    enc = {s: tok.encode(s) for s in probes}
    return table, enc


# class names for the template probes: punctuation inside words (hyphen, apostrophe), several
# words, digits, capitals, and long words the BPE merge loop builds from many merges
PROBE_NAMES = ["dog", "golden retriever", "jack-o'-lantern", "potter's wheel", "T-shirt", "hen-of-the-woods",
               "Granny Smith", "class123", "African elephant", "internationalization", "photographs",
               "unbelievably embroidered", "3D printer", "rock beauty", "Yorkshire terrier", "spider web",
               "crossword puzzle", "car mirror", "Band Aid", "water ouzel"]
EXTRA_PROBES = ["  multiple   spaces  and\ttabs  ", "semicolons; colons: dashes -- and (parens)",
                "&amp; html escapes &lt;b&gt;", "a photo of a {}, a type of pet.", "ALL CAPS SHOUTING!!!",
                "mixed123digits456and789words", "it's they're we've I'm you'll he'd", "e.g. i.e. etc.",
                "comma,separated,values", "question? exclamation! period."]


def template_probes():
    """Every prompt template the reference ships (trainers/imagenet_templates.py
    IMAGENET_TEMPLATES + IMAGENET_TEMPLATES_SELECT, trainers/zsclip.py CUSTOM_TEMPLATES), each
    filled with one of PROBE_NAMES in turn, plus EXTRA_PROBES."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("ref_imagenet_templates",
                                                  os.path.join(REF, "trainers", "imagenet_templates.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    import trainers.zsclip as zs
    temps = list(m.IMAGENET_TEMPLATES) + list(m.IMAGENET_TEMPLATES_SELECT) + sorted(set(zs.CUSTOM_TEMPLATES.values()))
    out = []
    for i, t in enumerate(temps):
        s = t.format(PROBE_NAMES[i % len(PROBE_NAMES)])
        if s not in out:
            out.append(s)
    return out + EXTRA_PROBES


def save(name, meta, arrays):
    np.savez_compressed(os.path.join(HERE, name + ".npz"), meta=json.dumps(meta), **arrays)
    print("wrote", name, {k: v.shape for k, v in arrays.items()})


def run_cocoop_headline(arch, n_cls, batch, ctx_init, n_ctx, chunk=100, fp16_values=False):
    """run_cocoop at the benchmark's size (ViT-B/16, C = 1,000, B = 8), where the reference's
    one-shot autograd graph would hold ~40 GB of text activations per image: the same
    reference modules and the same arithmetic as CustomCLIP.forward (cocoop.py:235-260) --
    image_encoder, prompt_learner (meta_net, ctx_shifted, construct_prompts), text_encoder,
    normalize, logit_scale.exp() * imf @ txt^T, criterion -- with the text encoder evaluated
    over class chunks: the logits without a graph, then dlogits = d loss / d logits, then per
    (image, chunk) the text encoder re-run with a graph and back-propagated from its dlogits
    slice into the prompts, and finally prompts.backward(d prompts) into ctx and meta_net.
    Mathematically the reference's backward; only the fp32 summation order of the per-chunk
    gradient accumulation differs. fp16_values: on fp16-valued weights (the benchmark's, as a
    released checkpoint loads: PREC fp32s then runs split mode 2, CLIPK_F32S16)."""
    from clip.model import build_model
    import trainers.cocoop as cocoop
    tsd, digest = build_clip(arch, fp16_values)
    a = synth.ARCHS[arch]
    design = dict(DESIGN, trainer="CoCoOp")
    model = build_model(dict(tsd), design).float()
    cfg = make_cfg(a.image_resolution, cocoop=dict(N_CTX=n_ctx, CTX_INIT=ctx_init, PREC="fp32", USE_FOCAL_LOSS=False))
    names = synth.synthetic_classnames(n_cls)
    cc = cocoop.CustomCLIP(cfg, names, model)
    for n, p in cc.named_parameters():
        if "prompt_learner" not in n:
            p.requires_grad_(False)
    pl = cc.prompt_learner
    mn = synth.make_meta_net(a.embed_dim, a.transformer_width, seed=4)
    with torch.no_grad():
        for k, v in mn.items():
            dict(pl.named_parameters())[k].copy_(torch.from_numpy(v))
    ctx0 = pl.ctx.detach().clone().numpy()
    img = torch.from_numpy(synth.make_images(batch, a.image_resolution, seed=1))
    lbl = torch.from_numpy(synth.make_labels(batch, n_cls, seed=2))
    tok = cc.tokenized_prompts
    out = dict(arch=arch, digest=digest, n_cls=n_cls, batch=batch, n_ctx=pl.n_ctx, ctx_init=ctx_init, focal=0,
               chunked=chunk, fp16_values=bool(fp16_values))
    cc.train()
    imf_raw = cc.image_encoder(img.type(cc.dtype))
    imf = imf_raw / imf_raw.norm(dim=-1, keepdim=True)
    prompts = cc.prompt_learner(imf)  # (batch, n_cls, n_tkn, dim), graph to ctx / meta_net
    scale = cc.logit_scale.exp()

    def chunk_logits(b, c0, c1, p):
        tf = cc.text_encoder(p, tok[c0:c1])
        tf = tf / tf.norm(dim=-1, keepdim=True)
        return scale * imf[b].detach() @ tf.t()

    logits = torch.zeros(batch, n_cls)
    with torch.no_grad():
        for b in range(batch):
            for c0 in range(0, n_cls, chunk):
                c1 = min(c0 + chunk, n_cls)
                logits[b, c0:c1] = chunk_logits(b, c0, c1, prompts[b, c0:c1])
            print("logits image", b, flush=True)
    lg = logits.clone().requires_grad_(True)
    loss = cc.criterion(lg, lbl)
    (dlogits,) = torch.autograd.grad(loss, lg)
    dprompts = torch.zeros_like(prompts)
    for b in range(batch):
        for c0 in range(0, n_cls, chunk):
            c1 = min(c0 + chunk, n_cls)
            p = prompts[b, c0:c1].detach().requires_grad_(True)
            chunk_logits(b, c0, c1, p).backward(dlogits[b, c0:c1])
            dprompts[b, c0:c1] = p.grad
        print("backward image", b, flush=True)
    prompts.backward(dprompts)
    grads = {"grad_ctx": pl.ctx.grad.detach().clone().numpy()}
    for k, p in pl.named_parameters():
        if k.startswith("meta_net"):
            grads["grad_" + k] = p.grad.detach().clone().numpy()
    sgd_after_step(pl)
    arrays = dict(ctx0=ctx0, image_features=imf_raw.detach().numpy(), logits=logits.numpy(),
                  loss=np.asarray(loss.item(), np.float32), ctx_after_step=pl.ctx.detach().numpy(),
                  tokenized=tok.numpy().astype(np.int32), **grads)
    return out, arrays


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--full", action="store_true", help="also full-size ViT-B/L sets (slow)")
    ap.add_argument("--only", choices=["tokenizer", "headline", "headline_w16"],
                    help="tokenizer: the BPE probes alone; headline: the benchmark-size CoCoOp set alone "
                         "(ViT-B/16, C 1000, B 8: ~15 min on 8 threads)")
    args = ap.parse_args()
    torch.set_num_threads(8)
    _install_stubs()

    if args.only == "headline":
        m, a = run_cocoop_headline("ViT-B/16", 1000, 8, "a photo of a", 4)
        save("cocoop_vitb16_c1000_b8", m, a)
        return
    if args.only == "headline_w16":  # the benched configuration exactly: fp16-valued weights
        m, a = run_cocoop_headline("ViT-B/16", 1000, 8, "a photo of a", 4, fp16_values=True)
        save("cocoop_vitb16_c1000_b8_w16", m, a)
        return
    table, enc = tokenizer_table()
    pkg = os.path.join(REPO, "few-shot-prompt-learning-for-vision-language-models-in-imbalanced-datasets_amd")
    with open(os.path.join(pkg, "clip", "bpe_fallback.json"), "w") as f:
        json.dump(table, f, indent=0, sort_keys=True)
    with open(os.path.join(HERE, "tokenizer_probes.json"), "w") as f:
        json.dump(enc, f, indent=0, sort_keys=True)
    if args.only == "tokenizer":
        return

    lrs = lr_sequences()
    np.savez(os.path.join(HERE, "lr_schedule.npz"), ep10=lrs[10], ep50=lrs[50])

    shots = [4, 1, 2, 0, 3]  # includes a zero-count class (CoOp guards it, coop.py:341)
    for pos in ("end", "middle", "front"):
        for csc in (False, True):
            m, a = run_coop("tiny", 5, 3, 4, pos, csc, "ce")
            save(f"coop_tiny_{pos}_csc{int(csc)}_ce", m, a)
    m, a = run_coop("tiny", 5, 3, 4, "end", False, "focal", per_class=shots)
    save("coop_tiny_end_focal", m, a)
    m, a = run_coop("tiny", 5, 3, 4, "end", False, "simclr")
    save("coop_tiny_end_simclr", m, a)
    m, a = run_coop("tiny", 5, 3, 0, "end", False, "ce", ctx_init="a photo of a")
    save("coop_tiny_ctxinit_ce", m, a)
    m, a = run_coop("tiny-p8", 5, 3, 4, "end", False, "ce")
    save("coop_tinyp8_end_ce", m, a)
    m, a = run_cocoop("tiny", 5, 3, "a photo of a", 4, False)
    save("cocoop_tiny_ctxinit_ce", m, a)
    m, a = run_cocoop("tiny", 5, 3, "", 4, True, per_class=[4, 1, 2, 5, 3])
    save("cocoop_tiny_focal", m, a)

    if args.full:
        m, a = run_coop("ViT-B/32", 10, 2, 16, "end", False, "ce")
        save("coop_vitb32_c10", m, a)
        m, a = run_cocoop("ViT-B/16", 4, 2, "a photo of a", 4, False)
        save("cocoop_vitb16_c4", m, a)
        m, a = run_coop("ViT-B/16", 6, 2, 16, "end", False, "focal", per_class=[16, 16, 16, 1, 1, 1])
        save("coop_vitb16_c6_focal", m, a)
        m, a = run_coop("ViT-L/14", 4, 1, 16, "end", False, "ce")
        save("coop_vitl14_c4", m, a)
        m, a = run_cocoop("ViT-L/14@336px", 3, 1, "a photo of a", 4, False)
        save("cocoop_vitl14_336_c3", m, a)


if __name__ == "__main__":
    main()
