"""Golden vectors for the deep-prompt trainers, produced by running the
REFERENCE modules themselves on CPU in fp32: IVLP (trainers/independentVL.py CustomCLIP on
clip/model.py's ResidualAttentionBlock_IVLP), MaPLe (trainers/maple.py on
VisionTransformer_MaPLe / ResidualAttentionBlock_MaPLe) and the pieces of PromptSRC's loss
(trainers/promptsrc.py: prompted features, the frozen zero-shot features, fixed text
embeddings). Build container only (needs /root/reference):

    python tests/golden/make_golden_deep.py [--full]

Stand-ins, beyond make_golden.py's: ``timm`` (imported at independentVL.py:15 for the KD
teacher, unused here), ``load_clip_to_cpu`` of promptsrc.py (downloads CLIP: replaced by the
seeded synthetic build), ``.cuda()`` as identity (promptsrc.py:128-141). Deviations, each
because the reference cannot run the path as written on CPU fp32:
  * MaPLe: ``self.proj.half()`` (maple.py:146) meets fp32 ctx in every non-amp PREC and
    raises; the projection is converted back to fp32 after construction (its weights stay
    rounded to fp16), i.e. the amp path's math in fp32.
  * MaPLe: Transformer.forward's saved_features hook (model.py:364-366) cannot clone the
    list MaPLe's blocks carry; it is switched off (``transformer.init = False``).
  * PromptSRC: ``zero_shot_features @ fixed_embeddings.half().t()`` (promptsrc.py:204) raises
    in fp32; the zero-shot logits are formed in fp32 from fp16-rounded fixed embeddings, and
    the trainer's loss (promptsrc.py:296-323; LOGITS_LOSS_WEIGHT, absent from train.py's
    config, taken as 1) is evaluated on the reference's own features.
Trainable parameters get seeded values (normal, std 0.02) recorded in the fixture.
"""
from __future__ import annotations

import argparse
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as MG  # noqa: E402
from fsp_amd.clip import synth  # noqa: E402


def _stub_timm():
    sys.modules.setdefault("timm", types.ModuleType("timm"))


def _seed_params(module, names, seed):
    """normal(0, 0.02) from RandomState(seed), in `names` order (tests/deep_util.seeded_init
    regenerates the same values)."""
    rs = np.random.RandomState(seed)
    init = {}
    params = dict(module.named_parameters())
    with torch.no_grad():
        for n in names:
            p = params[n]
            v = rs.normal(0.0, 0.02, size=tuple(p.shape)).astype(np.float32)
            p.copy_(torch.from_numpy(v))
            init[n] = v
    return init


def _run(cc, trainable, img, lbl, loss_fn=None):
    cc.eval()
    with torch.no_grad():
        logits = cc(img) if loss_fn is None else None
    cc.train()
    loss = cc(img, lbl) if loss_fn is None else loss_fn()
    loss.backward()
    params = dict(cc.named_parameters())
    grads = {"grad_" + n: params[n].grad.detach().clone().numpy() for n in trainable}
    return logits, loss, grads


def _trainable(cc):
    """The reference's selection (independentVL.py:385-391, maple.py:276-285)."""
    out = []
    for n, p in cc.named_parameters():
        on = ("prompt_learner" in n and "ZS_image_encoder" not in n) or "VPT" in n
        p.requires_grad_(on)
        if on:
            out.append(n)
    return out


def run_ivlp(arch, n_cls, batch, n_ctx_t, n_ctx_v, depth_t, depth_v, ctx_init="a photo of a"):
    from clip.model import build_model
    import trainers.independentVL as ivlp
    tsd, digest = MG.build_clip(arch)
    a = synth.ARCHS[arch]
    design = {"trainer": "IVLP", "vision_depth": depth_v, "language_depth": depth_t,
              "vision_ctx": n_ctx_v, "language_ctx": n_ctx_t}
    model = build_model(dict(tsd), design).float()
    cfg = MG.make_cfg(a.image_resolution)
    cfg.TRAINER["IVLP"] = MG.Cfg(N_CTX_TEXT=n_ctx_t, N_CTX_VISION=n_ctx_v, CTX_INIT=ctx_init, PREC="fp32",
                                 PROMPT_DEPTH_TEXT=depth_t, PROMPT_DEPTH_VISION=depth_v, USE_FOCAL_LOSS=False,
                                 SIMCLR_ALPHA=0.0)
    cc = ivlp.CustomCLIP(cfg, synth.synthetic_classnames(n_cls), model)
    trainable = _trainable(cc)
    init = _seed_params(cc, [n for n in trainable if "VPT" in n], seed=11)
    init["prompt_learner.ctx"] = cc.prompt_learner.ctx.detach().clone().numpy()
    img = torch.from_numpy(synth.make_images(batch, a.image_resolution, seed=1))
    lbl = torch.from_numpy(synth.make_labels(batch, n_cls, seed=2))
    logits, loss, grads = _run(cc, trainable, img, lbl)
    meta = dict(arch=arch, digest=digest, n_cls=n_cls, batch=batch, n_ctx_text=n_ctx_t, n_ctx_vision=n_ctx_v,
                depth_text=depth_t, depth_vision=depth_v, ctx_init=ctx_init, trainable=trainable)
    arrays = {"init_" + k: v for k, v in init.items()}
    arrays.update(logits=logits.numpy(), loss=np.asarray(loss.item(), np.float32),
                  tokenized=cc.tokenized_prompts.numpy().astype(np.int32), **grads)
    return meta, arrays


def run_maple(arch, n_cls, batch, n_ctx, depth, ctx_init="a photo of a"):
    from clip.model import build_model
    import trainers.maple as maple
    tsd, digest = MG.build_clip(arch)
    a = synth.ARCHS[arch]
    design = {"trainer": "MaPLe", "vision_depth": depth, "language_depth": depth, "vision_ctx": n_ctx,
              "language_ctx": n_ctx, "maple_length": n_ctx}
    model = build_model(dict(tsd), design).float()
    cfg = MG.make_cfg(a.image_resolution)
    cfg.TRAINER["MAPLE"] = MG.Cfg(N_CTX=n_ctx, CTX_INIT=ctx_init, PREC="fp32", PROMPT_DEPTH=depth,
                                  USE_FOCAL_LOSS=False)
    cc = maple.CustomCLIP(cfg, synth.synthetic_classnames(n_cls), model)
    cc.prompt_learner.proj.float()  # see the module docstring
    # Transformer.forward's saved_features side effect (model.py:364-366) calls .clone() on
    # the list the MaPLe blocks pass along and raises on the first forward; it is off once
    # `init` is False (the features it saves are unused by the trainers)
    cc.text_encoder.transformer.init = False
    cc.image_encoder.transformer.init = False
    trainable = _trainable(cc)
    pl = cc.prompt_learner
    init = _seed_params(cc, [n for n in trainable if "compound" in n or n.endswith("proj.weight")
                             or n.endswith("proj.bias")], seed=12)
    with torch.no_grad():  # the reference's proj weights are fp16 values
        pl.proj.weight.copy_(pl.proj.weight.half().float())
        pl.proj.bias.copy_(pl.proj.bias.half().float())
    seeded = [n for n in trainable if "compound" in n or n.endswith("proj.weight") or n.endswith("proj.bias")]
    init["prompt_learner.ctx"] = pl.ctx.detach().clone().numpy()
    img = torch.from_numpy(synth.make_images(batch, a.image_resolution, seed=1))
    lbl = torch.from_numpy(synth.make_labels(batch, n_cls, seed=2))
    logits, loss, grads = _run(cc, trainable, img, lbl)
    # the [768, 512] projection matrices are not stored: seeded_init() regenerates them (seed
    # 12, this order; proj's rounded to fp16); of their gradients the first 32 rows are kept
    big = [n for n in init if init[n].size > 65536]
    for n in big:
        init.pop(n)
    for n in list(grads):
        if grads[n].size > 65536:
            grads[n + ".rows32"] = grads.pop(n)[:32]
    meta = dict(arch=arch, digest=digest, n_cls=n_cls, batch=batch, n_ctx=n_ctx, depth=depth, ctx_init=ctx_init,
                trainable=trainable, seeded=seeded, seed=12, half_rounded=["prompt_learner.proj.weight",
                                                                          "prompt_learner.proj.bias"])
    arrays = {"init_" + k: v for k, v in init.items()}
    arrays.update(logits=logits.numpy(), loss=np.asarray(loss.item(), np.float32),
                  tokenized=pl.tokenized_prompts.numpy().astype(np.int32), **grads)
    return meta, arrays


def run_promptsrc(arch, n_cls, batch, n_ctx_t, n_ctx_v, depth_t, depth_v, ctx_init="a photo of a"):
    from clip.model import build_model
    import trainers.promptsrc as psrc
    import torch.nn.functional as F
    tsd, digest = MG.build_clip(arch)
    a = synth.ARCHS[arch]

    def load_clip_to_cpu(cfg, zero_shot_model=False):
        d = {"trainer": "IVLP", "vision_depth": 0 if zero_shot_model else depth_v,
             "language_depth": 0 if zero_shot_model else depth_t,
             "vision_ctx": 0 if zero_shot_model else n_ctx_v, "language_ctx": 0 if zero_shot_model else n_ctx_t}
        return build_model(dict(tsd), d)

    psrc.load_clip_to_cpu = load_clip_to_cpu
    torch.Tensor.cuda = lambda self, *a, **k: self
    torch.nn.Module.cuda = lambda self, *a, **k: self
    model = load_clip_to_cpu(None).float()
    cfg = MG.make_cfg(a.image_resolution)
    cfg.OPTIM = MG.Cfg(MAX_EPOCH=20)
    cfg.TRAINER["PROMPTSRC"] = MG.Cfg(N_CTX_TEXT=n_ctx_t, N_CTX_VISION=n_ctx_v, CTX_INIT=ctx_init, PREC="fp32",
                                      PROMPT_DEPTH_TEXT=depth_t, PROMPT_DEPTH_VISION=depth_v,
                                      TEXT_LOSS_WEIGHT=25, IMAGE_LOSS_WEIGHT=10, GPA_MEAN=15, GPA_STD=1)
    cc = psrc.CustomCLIP(cfg, synth.synthetic_classnames(n_cls), model)
    trainable = _trainable(cc)
    init = _seed_params(cc, [n for n in trainable if "VPT" in n], seed=13)
    init["prompt_learner.ctx"] = cc.prompt_learner.ctx.detach().clone().numpy()
    img = torch.from_numpy(synth.make_images(batch, a.image_resolution, seed=1))
    lbl = torch.from_numpy(synth.make_labels(batch, n_cls, seed=2))
    pl = cc.prompt_learner
    cc.train()
    # the reference CustomCLIP.forward, training branch (promptsrc.py:183-213), up to the
    # fp16 matmul that raises in fp32: the same features from the reference's own modules
    prompts = pl()
    txt = cc.text_encoder(prompts, cc.tokenized_prompts)
    imf = cc.image_encoder(img)
    imf_n = imf / imf.norm(dim=-1, keepdim=True)
    txt_n = txt / txt.norm(dim=-1, keepdim=True)
    scale = cc.logit_scale.exp()
    logits = scale * imf_n @ txt_n.t()
    fixed = pl.fixed_embeddings
    fixed_n = fixed / fixed.norm(dim=-1, keepdim=True)
    with torch.no_grad():
        zs = pl.ZS_image_encoder(img)
        zs_n = zs / zs.norm(dim=-1, keepdim=True)
        zs_logits = scale * zs_n @ fixed_n.half().float().t()
    loss_ce = F.cross_entropy(logits, lbl)
    l_text = F.l1_loss(txt_n, fixed_n, reduction="mean") * 25
    l_img = F.l1_loss(imf_n, zs_n, reduction="mean") * 10
    l_log = F.kl_div(F.log_softmax(logits, dim=1), F.log_softmax(zs_logits, dim=1), reduction="sum",
                     log_target=True) / logits.numel()
    loss = loss_ce + (l_log + l_text + l_img)
    loss.backward()
    params = dict(cc.named_parameters())
    grads = {"grad_" + n: params[n].grad.detach().clone().numpy() for n in trainable}
    gauss = psrc.PromptSRC.get_gauss(None, 15, 1)
    gw = np.array([gauss(x) for x in range(1, 21)])
    meta = dict(arch=arch, digest=digest, n_cls=n_cls, batch=batch, n_ctx_text=n_ctx_t, n_ctx_vision=n_ctx_v,
                depth_text=depth_t, depth_vision=depth_v, ctx_init=ctx_init, trainable=trainable)
    arrays = {"init_" + k: v for k, v in init.items()}
    arrays.update(logits=logits.detach().numpy(), loss=np.asarray(loss.item(), np.float32),
                  loss_ce=np.asarray(loss_ce.item(), np.float32), zs_logits=zs_logits.numpy(),
                  fixed_embeddings=fixed.detach().numpy(), zs_image_features=zs.numpy(),
                  tokenized=cc.tokenized_prompts.numpy().astype(np.int32), gpa_weights=gw / gw.sum(), **grads)
    return meta, arrays


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--full", action="store_true")
    ap.add_argument("--maple", action="store_true", help="only the MaPLe fixture")
    args = ap.parse_args()
    torch.set_num_threads(8)
    MG._install_stubs()
    _stub_timm()
    if args.maple and not args.full:
        m, a = run_maple("ViT-B/32", 3, 2, 2, 9)
        MG.save("maple_vitb32_c3", m, a)
        return
    m, a = run_ivlp("tiny4", 5, 3, 4, 3, 3, 4)
    MG.save("ivlp_tiny4", m, a)
    m, a = run_ivlp("tiny4", 4, 2, 2, 2, 1, 0, ctx_init="")  # shallow text, no vision prompts
    MG.save("ivlp_tiny4_shallow", m, a)
    m, a = run_promptsrc("tiny4", 5, 3, 4, 4, 3, 3)
    MG.save("promptsrc_tiny4", m, a)
    if args.full or args.maple:
        m, a = run_maple("ViT-B/32", 3, 2, 2, 9)
        MG.save("maple_vitb32_c3", m, a)
    if args.full:
        m, a = run_ivlp("ViT-B/16", 3, 2, 4, 4, 9, 9)
        MG.save("ivlp_vitb16_c3", m, a)


if __name__ == "__main__":
    main()
