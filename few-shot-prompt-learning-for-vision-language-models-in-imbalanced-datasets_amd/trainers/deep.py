"""Deep (multi-layer) vision-language prompting on the MI355X-native path:
IVLP (``PromptSRC/trainers/independentVL.py``), MaPLe (``trainers/maple.py``) and PromptSRC
(``trainers/promptsrc.py``) -- same registry names, cfg keys (TRAINER.{IVLP,MAPLE,PROMPTSRC}.*)
and trainable-parameter names as the reference's CustomCLIPs, so their checkpoints load.

Per step: the class prompts (ctx spliced into the token embeddings, PromptAssembleFn) go
through the native text encoder with deep prompts replacing tokens 1..n_ctx before layers
1..depth-1 (DeepTextEncodeFn; model.py:242-252, 313-328); the images through the prompted
ViT (PromptedVisionFn: n_vpt prompt rows after the image tokens, replaced again before layers
1..depth-1, model.py:234-241, 299-312, 413-420, 465-472), whose input-grad backward reaches
every visual prompt. Prompt tokens are rounded to fp16 values as the reference's ``.half()``
does (gradient passed straight through). The [B, C] cosine head and the losses on it are
composed from torch ops on a few KB (the image side needs its gradient here).
"""
from __future__ import annotations

import copy
import math
import os.path as osp

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from ..engine.registry import TRAINER_REGISTRY
from ..engine.trainer import TrainerX, load_clip
from ..engine.optim import build_optimizer, build_lr_scheduler
from ..engine.metrics import LossSummary
from ..clip.model import TextEncodeFn, DeepTextEncodeFn, PromptedVisionFn
from ._fns import PromptAssembleFn, CrossEntropyFn
from .losses import focal_alpha
from .prompt_base import init_prompts, grads_finite


def half_values(x):
    """x rounded to fp16 values (the reference's prompt ``.half()``), identity gradient."""
    return x + (x.half().float() - x).detach()


class _Block(nn.Module):
    """Stands in for a ResidualAttentionBlock_IVLP: holds its VPT_shallow prompt only."""


class DeepPrompts(nn.Module):
    """The prompt parameters an encoder of the reference carries, under its names:
    ``transformer.resblocks.{i}.VPT_shallow`` for i = 1..depth-1 (model.py:210-221) and, for
    the ViT with depth >= 1, ``VPT`` (model.py:377-386). The frozen weights stay in the
    native encoders."""

    def __init__(self, n_layers, depth, n_ctx, width, first=False):
        super().__init__()
        self.depth, self.n_ctx = depth, n_ctx
        self.transformer = nn.Module()
        self.transformer.resblocks = nn.ModuleList([_Block() for _ in range(n_layers)])
        for i in range(1, min(depth, n_layers)):
            v = torch.empty(n_ctx, width)
            nn.init.normal_(v, std=0.02)
            self.transformer.resblocks[i].VPT_shallow = nn.Parameter(v)
        if first and depth >= 1:
            v = torch.empty(n_ctx, width)
            nn.init.normal_(v, std=0.02)
            self.VPT = nn.Parameter(v)

    def deep(self):
        ps = [b.VPT_shallow for b in self.transformer.resblocks if hasattr(b, "VPT_shallow")]
        return torch.stack([half_values(p) for p in ps]) if ps else None

    def first(self):
        return half_values(self.VPT) if hasattr(self, "VPT") else None


class VLPromptLearner(nn.Module):
    """independentVL.py:195-254 / promptsrc.py:73-168: a shared text context (CTX_INIT used
    when N_CTX <= 4), token_prefix / token_suffix buffers; ``assemble()`` is the native splice."""

    def __init__(self, sec, classnames, clip_model, cfg):
        super().__init__()
        clip_imsize = clip_model.visual.input_resolution
        assert cfg.INPUT.SIZE[0] == clip_imsize, \
            f"cfg_imsize ({cfg.INPUT.SIZE[0]}) must equal to clip_imsize ({clip_imsize})"
        truncate = cfg.get("NATIVE", {}).get("TRUNCATE_PROMPTS", True)
        shared = cfg.get("NATIVE", {}).get("SHARED_PREFIX", True)
        n_ctx = sec.get("N_CTX_TEXT", sec.get("N_CTX"))
        ctx_vectors, self.prompt_prefix = init_prompts(self, classnames, clip_model, n_ctx, sec.CTX_INIT, "end",
                                                       False, truncate, shared, None, vl_init=True)
        self.ctx = nn.Parameter(ctx_vectors)

    def assemble(self):
        return PromptAssembleFn.apply(self.ctx, None, self.layout)

    def forward(self):
        ctx = self.ctx.unsqueeze(0).expand(self.n_cls, -1, -1)
        return torch.cat([self.token_prefix, ctx, self.token_suffix], dim=1)


class _DeepCLIP(nn.Module):
    """Shared forward of the IVLP / PromptSRC / MaPLe CustomCLIPs on the native encoders."""

    def _setup(self, clip_model):
        object.__setattr__(self, "clip", clip_model)  # frozen native encoders: not submodules
        self.logit_scale = clip_model.logit_scale
        self.logit_scale_value = clip_model.logit_scale_value
        self.dtype = clip_model.dtype

    # prompt sources, overridden by MaPLe
    def _text_deep(self):
        return self.text_encoder.deep()

    def _vision_prompts(self):
        return self.image_encoder.first(), self.image_encoder.deep()

    def text_features(self):
        pl = self.prompt_learner
        x0 = pl.assemble()
        shape = pl.layout.shape(1)
        deep = self._text_deep()
        if deep is None:
            return TextEncodeFn.apply(x0, self.clip.text, shape)
        return DeepTextEncodeFn.apply(x0, deep, self.clip.text, shape)

    def image_features(self, image):
        vpt, deep = self._vision_prompts()
        if vpt is None:
            return self.clip.visual(image)
        return PromptedVisionFn.apply(vpt, deep, image, self.clip.visual)

    def cached_text_features(self):
        """Eval without autograd: encode the class prompts once per parameter version."""
        key = tuple((p.data_ptr(), p._version, getattr(p, "_clipk_gen", 0)) for p in self.parameters())
        cache = getattr(self, "_txt_cache", None)
        if cache is None or cache[0] != key:
            cache = self._txt_cache = (key, self.text_features())
        return cache[1]

    def train(self, mode=True):
        self._txt_cache = None
        return super().train(mode)

    def features(self, image):
        """L2-normalised (image, text) features and logit_scale * cos logits."""
        if not self.training and not torch.is_grad_enabled():
            txt = self.cached_text_features()
        else:
            txt = self.text_features()
        img = F.normalize(self.image_features(image), dim=-1)
        txt = F.normalize(txt, dim=-1)
        return img, txt, self.logit_scale_value * img @ txt.t()


def _criterion(sec, n_cls, per_class):
    if sec.get("USE_FOCAL_LOSS", False):
        print(">> Use Focal Loss!")
        return focal_alpha(per_class, n_cls, zero_guard=True), True
    print(">> Use Cross Entropy Loss!")
    return None, False


class IVLPCustomCLIP(_DeepCLIP):
    """independentVL.py:257-333 (CustomCLIP): CE / focal on cosine logits, optional image
    NT-Xent (SIMCLR_ALPHA, ImageNTXentLoss on two views, independentVL.py:73-112)."""

    def __init__(self, cfg, classnames, clip_model, sec):
        super().__init__()
        self._setup(clip_model)
        self.prompt_learner = VLPromptLearner(sec, classnames, clip_model, cfg)
        self.tokenized_prompts = self.prompt_learner.tokenized_prompts
        a = clip_model.arch
        assert sec.PROMPT_DEPTH_TEXT >= 1, "In Independent VL prompting, Language prompt depth should be >=1"
        self.text_encoder = DeepPrompts(a.transformer_layers, sec.PROMPT_DEPTH_TEXT, sec.N_CTX_TEXT,
                                        a.transformer_width)
        self.image_encoder = DeepPrompts(a.vision_layers, sec.PROMPT_DEPTH_VISION, sec.N_CTX_VISION, a.vision_width,
                                         first=True)
        alpha, self.focal = _criterion(sec, len(classnames), cfg.DATASET.get("PER_CLASS_SHOTS", None))
        self.alpha = torch.tensor(alpha, dtype=torch.float32, device=clip_model.logit_scale.device) \
            if alpha is not None else None
        self.simclr_alpha = float(sec.get("SIMCLR_ALPHA", 0.0))

    def criterion(self, logits, y):
        return CrossEntropyFn.apply(logits, y, self.alpha, 2.0, self.focal)

    def forward(self, image1, label=None, image2=None):
        img, _, logits = self.features(image1)
        if not self.training:
            return logits
        total = self.criterion(logits, label) if label is not None else 0.0
        if image2 is not None and self.simclr_alpha > 0.0:
            img2 = F.normalize(self.image_features(image2), dim=-1)
            total = total + self.simclr_alpha * image_ntxent(img, img2)
        return total


def image_ntxent(z1, z2, temperature=0.07):
    """ImageNTXentLoss (independentVL.py:73-112), vectorised: positives z1[i] <-> z2[i]."""
    z = torch.cat([F.normalize(z1, dim=1), F.normalize(z2, dim=1)], 0)
    n2 = z.shape[0]
    n = n2 // 2
    sim = z @ z.t() / temperature
    idx = torch.arange(n2, device=z.device)
    pos = torch.cat([idx[:n] + n, idx[n:] - n])
    keep = (idx[None, :] != idx[:, None]) & (idx[None, :] != pos[:, None])
    out = torch.cat([sim[idx, pos][:, None], sim[keep].view(n2, n2 - 2)], 1)
    return F.cross_entropy(out, torch.zeros(n2, dtype=torch.long, device=z.device))


class _DeepTrainer(TrainerX):
    """Common trainer body (independentVL.py:337-589, maple.py:258-367, promptsrc.py:217-419)."""

    SEC = ""
    MODEL_NAME = ""

    @property
    def sec(self):
        return self.cfg.TRAINER[self.SEC]

    def check_cfg(self, cfg):
        assert cfg.TRAINER[self.SEC].PREC in ["fp16", "fp32", "amp", "bf16", "fp32s"]

    def _vision_trains(self):
        raise NotImplementedError

    def _make_model(self, classnames, clip_model):
        raise NotImplementedError

    def build_model(self):
        cfg = self.cfg
        classnames = self.dm.dataset.classnames
        clip_model = load_clip(cfg, self.sec.PREC, self.device, vision_grad=self._vision_trains())
        print(f"Building custom CLIP ({self.SEC})")
        self.model = self._make_model(classnames, clip_model).to(self.device)
        # the reference's selection: prompt_learner.* and every *VPT* (independentVL.py:385-391)
        for name, p in self.model.named_parameters():
            p.requires_grad_(("prompt_learner" in name) or ("VPT" in name))
        enabled = sorted(n for n, p in self.model.named_parameters() if p.requires_grad)
        print(f"Parameters to be updated: {set(enabled)}")
        if cfg.MODEL.INIT_WEIGHTS:
            self.load_pretrained_weights(self.model, cfg.MODEL.INIT_WEIGHTS)
        self.optim = build_optimizer(self.model, cfg.OPTIM)
        self.sched = build_lr_scheduler(self.optim, cfg.OPTIM)
        self.register_model(self.MODEL_NAME, self.model, self.optim, self.sched)

    def parse_batch_train(self, batch):
        return batch["img"].to(self.device), batch["label"].to(self.device)

    def _step(self, loss, batch, n_local):
        self.optim.zero_grad()
        w = self.batch_weight(batch, n_local)
        (loss * w if w != 1.0 else loss).backward()
        self.allreduce_grads(self.model)
        if self.sec.PREC != "amp" or grads_finite(self.model):
            self.optim.step()

    def load_model(self, directory, epoch=None):
        """independentVL.py:566-589: token_prefix / token_suffix dropped, strict=False (the
        reference checkpoints also hold the frozen CLIP weights; they are ignored here)."""
        if not directory:
            print("Note that load_model() is skipped as no pretrained model is given")
            return
        model_file = "model-best.pth.tar" if epoch is None else f"model.pth.tar-{epoch}"
        for name in self.get_model_names():
            model_path = osp.join(directory, name, model_file)
            if not osp.exists(model_path):
                raise FileNotFoundError(f'Model not found at "{model_path}"')
            ckpt = self.load_checkpoint(model_path)
            sd = ckpt["state_dict"]
            sd.pop("prompt_learner.token_prefix", None)
            sd.pop("prompt_learner.token_suffix", None)
            own = self._models[name].state_dict()
            sd = {k: v for k, v in sd.items() if k in own}
            print(f'Loading weights to {name} from "{model_path}" (epoch = {ckpt["epoch"]})')
            self._models[name].load_state_dict(sd, strict=False)


@TRAINER_REGISTRY.register()
class IVLP(_DeepTrainer):
    """independentVL.py:337-589. Batches: {"img", "label"}; SimCLR {"img1", "img2", "label"};
    mixup {"img", "y_a", "y_b", "lam"} (parse_batch_train, independentVL.py:435-460). USE_KD
    needs a pretrained timm teacher (independentVL.py:360-365) and is refused."""

    SEC, MODEL_NAME = "IVLP", "VLPromptLearner"

    def _vision_trains(self):
        return self.sec.PROMPT_DEPTH_VISION >= 1

    def _make_model(self, classnames, clip_model):
        if self.sec.get("USE_KD", False):
            raise NotImplementedError("TRAINER.IVLP.USE_KD: the distillation teacher is a pretrained timm "
                                      "download (independentVL.py:360-365), unavailable on this path")
        return IVLPCustomCLIP(self.cfg, classnames, clip_model, self.sec)

    def parse_batch_train(self, batch):
        if "y_a" in batch and "y_b" in batch and "lam" in batch:
            return batch["img"].to(self.device), None, None, (batch["y_a"].to(self.device),
                                                              batch["y_b"].to(self.device), float(batch["lam"]))
        if "img1" in batch and "img2" in batch:
            return batch["img1"].to(self.device), batch["label"].to(self.device), batch["img2"].to(self.device), None
        return batch["img"].to(self.device), batch["label"].to(self.device), None, None

    def forward_backward(self, batch):
        image1, label, image2, mix = self.parse_batch_train(batch)
        m = self.model
        if mix is not None:
            y_a, y_b, lam = mix
            _, _, logits = m.features(image1)
            loss = lam * m.criterion(logits, y_a) + (1 - lam) * m.criterion(logits, y_b)
        else:
            loss = m(image1, label, image2)
        self._step(loss, batch, image1.shape[0])
        out = LossSummary()
        out["loss"] = loss
        if (self.batch_idx + 1) == self.num_batches:
            self.update_lr()
        return out


class MultiModalPromptLearner(nn.Module):
    """maple.py:112-204: shared ctx (N_CTX, CTX_INIT when N_CTX <= 4), its projection to the
    vision width (proj, fp16-rounded initial weights as the reference's ``.half()``),
    compound text prompts for layers 1..depth-1 and their per-layer projections."""

    def __init__(self, cfg, classnames, clip_model):
        super().__init__()
        sec = cfg.TRAINER.MAPLE
        assert sec.PROMPT_DEPTH >= 1, "PROMPT_DEPTH must be >= 1"
        self.compound_prompts_depth = sec.PROMPT_DEPTH
        a = clip_model.arch
        truncate = cfg.get("NATIVE", {}).get("TRUNCATE_PROMPTS", True)
        shared = cfg.get("NATIVE", {}).get("SHARED_PREFIX", True)
        assert cfg.INPUT.SIZE[0] == clip_model.visual.input_resolution
        ctx_vectors, self.prompt_prefix = init_prompts(self, classnames, clip_model, sec.N_CTX, sec.CTX_INIT, "end",
                                                       False, truncate, shared, None, vl_init=True)
        W, D = a.transformer_width, a.vision_width
        self.proj = nn.Linear(W, D)
        with torch.no_grad():
            self.proj.weight.copy_(self.proj.weight.half().float())
            self.proj.bias.copy_(self.proj.bias.half().float())
        self.ctx = nn.Parameter(ctx_vectors)
        self.compound_prompts_text = nn.ParameterList(
            [nn.Parameter(torch.empty(sec.N_CTX, W).normal_(std=0.02)) for _ in range(sec.PROMPT_DEPTH - 1)])
        single = nn.Linear(W, D)
        self.compound_prompt_projections = nn.ModuleList([copy.deepcopy(single) for _ in range(sec.PROMPT_DEPTH - 1)])
        dev = clip_model.logit_scale.device
        self.to(dev)

    def assemble(self):
        return PromptAssembleFn.apply(self.ctx, None, self.layout)

    def forward(self):
        ctx = self.ctx.unsqueeze(0).expand(self.n_cls, -1, -1)
        prompts = torch.cat([self.token_prefix, ctx, self.token_suffix], dim=1)
        visual_deep = [layer(self.compound_prompts_text[i]) for i, layer in enumerate(self.compound_prompt_projections)]
        return prompts, self.proj(self.ctx), self.compound_prompts_text, visual_deep


class MaPLeCustomCLIP(_DeepCLIP):
    """maple.py:206-256."""

    def __init__(self, cfg, classnames, clip_model):
        super().__init__()
        self._setup(clip_model)
        self.prompt_learner = MultiModalPromptLearner(cfg, classnames, clip_model)
        self.tokenized_prompts = self.prompt_learner.tokenized_prompts
        alpha, self.focal = _criterion(cfg.TRAINER.MAPLE, len(classnames), cfg.DATASET.get("PER_CLASS_SHOTS", None))
        self.alpha = torch.tensor(alpha, dtype=torch.float32, device=clip_model.logit_scale.device) \
            if alpha is not None else None

    def _text_deep(self):
        ps = list(self.prompt_learner.compound_prompts_text)
        return torch.stack([half_values(p) for p in ps]) if ps else None

    def _vision_prompts(self):
        pl = self.prompt_learner
        shared = half_values(pl.proj(pl.ctx))
        deep = [half_values(layer(pl.compound_prompts_text[i])) for i, layer in enumerate(pl.compound_prompt_projections)]
        return shared, (torch.stack(deep) if deep else None)

    def forward(self, image, label=None):
        _, _, logits = self.features(image)
        if self.training and label is not None:
            return CrossEntropyFn.apply(logits, label, self.alpha, 2.0, self.focal)
        return logits


@TRAINER_REGISTRY.register()
class MaPLe(_DeepTrainer):
    """maple.py:258-367."""

    SEC, MODEL_NAME = "MAPLE", "MultiModalPromptLearner"

    def _vision_trains(self):
        return True

    def _make_model(self, classnames, clip_model):
        return MaPLeCustomCLIP(self.cfg, classnames, clip_model)

    def forward_backward(self, batch):
        image, label = self.parse_batch_train(batch)
        loss = self.model(image, label)
        self._step(loss, batch, image.shape[0])
        out = LossSummary()
        out["loss"] = loss
        if (self.batch_idx + 1) == self.num_batches:
            self.update_lr()
        return out


class PromptSRCCustomCLIP(_DeepCLIP):
    """promptsrc.py:171-213: IVLP prompts plus the frozen CLIP's zero-shot text embeddings of
    "a photo of a {class}." (``fixed_embeddings``, computed once) and image features (the
    same weights without prompts: the native plain ViT)."""

    def __init__(self, cfg, classnames, clip_model):
        super().__init__()
        sec = cfg.TRAINER.PROMPTSRC
        self._setup(clip_model)
        self.prompt_learner = VLPromptLearner(sec, classnames, clip_model, cfg)
        self.tokenized_prompts = self.prompt_learner.tokenized_prompts
        a = clip_model.arch
        self.text_encoder = DeepPrompts(a.transformer_layers, sec.PROMPT_DEPTH_TEXT, sec.N_CTX_TEXT,
                                        a.transformer_width)
        self.image_encoder = DeepPrompts(a.vision_layers, sec.PROMPT_DEPTH_VISION, sec.N_CTX_VISION, a.vision_width,
                                         first=True)
        self.total_epochs = cfg.OPTIM.MAX_EPOCH
        self.n_cls = len(classnames)
        from .zsclip import encode_prompts
        # a plain attribute, as in the reference (not part of the state dict); stored
        # normalised (the forward normalises it again, promptsrc.py:197)
        self.prompt_learner.fixed_embeddings = encode_prompts(
            clip_model, ["a photo of a {}.".format(n.replace("_", " ")) for n in classnames],
            clip_model.logit_scale.device)

    def forward(self, image, label=None):
        img, txt, logits = self.features(image)
        if not self.prompt_learner.training:
            return logits
        fixed = F.normalize(self.prompt_learner.fixed_embeddings, dim=-1)
        with torch.no_grad():
            zs = F.normalize(self.clip.visual(image), dim=-1)
            zs_logits = self.logit_scale_value * zs @ fixed.half().float().t()
        return CrossEntropyFn.apply(logits, label, None, 0.0, False), txt, fixed, zs, img, zs_logits, logits


@TRAINER_REGISTRY.register()
class PromptSRC(_DeepTrainer):
    """promptsrc.py:217-419: CE + the self-regulating losses (L1 to the frozen text / image
    features, KL of the logits to the zero-shot logits) and Gaussian prompt aggregation (GPA)
    over epochs."""

    SEC, MODEL_NAME = "PROMPTSRC", "VLPromptLearner"

    def _vision_trains(self):
        return self.sec.PROMPT_DEPTH_VISION >= 1

    def _make_model(self, classnames, clip_model):
        return PromptSRCCustomCLIP(self.cfg, classnames, clip_model)

    def build_model(self):
        super().build_model()
        n, mean, std = self.cfg.OPTIM.MAX_EPOCH, self.sec.GPA_MEAN, self.sec.GPA_STD
        gauss = np.array([(1 / (std * np.sqrt(2 * np.pi))) * np.exp(-0.5 * ((a - mean) / std) ** 2)
                          for a in range(1, n + 1)])
        self.gauss = gauss / sum(gauss)
        self.step_counter = 1
        self.previous_model_gpa = None

    def forward_backward(self, batch):
        image, label = self.parse_batch_train(batch)
        s = self.sec
        loss_ce, txt, fixed, zs, img, zs_logits, logits = self.model(image, label)
        l_text = F.l1_loss(txt, fixed, reduction="mean") * s.TEXT_LOSS_WEIGHT
        l_img = F.l1_loss(img, zs, reduction="mean") * s.IMAGE_LOSS_WEIGHT
        l_logits = F.kl_div(F.log_softmax(logits, dim=1), F.log_softmax(zs_logits, dim=1), reduction="sum",
                            log_target=True) / logits.numel() * s.get("LOGITS_LOSS_WEIGHT", 1.0)
        loss = loss_ce + (l_logits + l_text + l_img)
        self._step(loss, batch, image.shape[0])
        out = LossSummary()
        out["loss"] = loss
        last = (self.batch_idx + 1) == self.num_batches
        if s.get("USE_GPA", True):
            if last:
                self.update_lr()
                self.step_counter += 1
                w = float(self.gauss[self.step_counter - 2])
                cur = {k: v.detach().clone() * w for k, v in self.model.state_dict().items()}
                if self.previous_model_gpa is None:
                    self.previous_model_gpa = cur
                else:
                    for k in cur:
                        self.previous_model_gpa[k] = self.previous_model_gpa[k] + cur[k]
            if self.step_counter == self.model.total_epochs + 1:
                print("Using GPA model for final inference...")
                self.model.load_state_dict(self.previous_model_gpa)
        elif last:
            self.update_lr()
        return out
