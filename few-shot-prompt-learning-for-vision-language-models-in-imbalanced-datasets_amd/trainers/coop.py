"""CoOp on the MI355X-native path — same registry name, cfg keys (TRAINER.COOP.*),
module contract and checkpoint format as ``PromptSRC/trainers/coop.py``.

Hot path per step (``CustomCLIP.forward_once``, coop.py:351-363):
  image_encoder (native ViT fwd) -> PromptAssembleFn (ctx spliced into the class
  token embeddings + pos) -> TextEncodeFn (native text transformer fwd, input-grad bwd)
  -> CosineLogitsFn -> CE / focal (fused kernel) or logit NT-Xent.
The text encoder runs once per step over the C class prompts (prompts are image
independent in CoOp), truncated to L = max EOT + 1 tokens (exact under the causal mask).
"""
from __future__ import annotations

import os.path as osp

import torch
import torch.nn as nn

from .. import dist
from ..engine.registry import TRAINER_REGISTRY
from ..engine.trainer import TrainerX, load_clip
from ..engine.optim import build_optimizer, build_lr_scheduler
from ..engine.metrics import compute_accuracy, LossSummary
from ..clip.model import TextEncodeFn
from ._fns import PromptAssembleFn, CosineLogitsFn
from .losses import CrossEntropyLoss, MultiClassFocalLoss, LogitsNTXentLoss, focal_alpha
from ._vision import ImageFeatureSchedule
from .prompt_base import init_prompts, TextShape, grads_finite


class TextEncoder(nn.Module):
    """API-compatible TextEncoder.forward(prompts [N,L,W], tokenized [N,77]) -> [N,E]
    (coop.py:186-205) on the native encoder; gradients flow to ``prompts``."""

    def __init__(self, clip_model):
        super().__init__()
        self.core = clip_model.text
        self.positional_embedding = clip_model.positional_embedding
        self.dtype = clip_model.dtype

    def forward(self, prompts, tokenized_prompts):
        N_, L77, W = prompts.shape
        eot = tokenized_prompts.argmax(dim=-1)
        L = int(eot.max().item()) + 1
        x0 = (prompts[:, :L] + self.positional_embedding[:L]).reshape(N_ * L, W).contiguous()
        rows = (torch.arange(N_, device=eot.device) * L + eot).to(torch.int32).to(prompts.device)
        return TextEncodeFn.apply(x0, self.core, TextShape(rows, nseq=N_, L=L))


class PromptLearner(nn.Module):
    """coop.py:207-296. forward() returns prompts [C,77,W] for API compatibility; the
    trainer's fast path uses ``assemble()`` (fused slot splice, no [C,77,W] concat)."""

    def __init__(self, cfg, classnames, clip_model, class_range=None):
        super().__init__()
        c = cfg.TRAINER.COOP
        clip_imsize = clip_model.visual.input_resolution
        cfg_imsize = cfg.INPUT.SIZE[0]
        assert cfg_imsize == clip_imsize, f"cfg_imsize ({cfg_imsize}) must equal to clip_imsize ({clip_imsize})"
        if c.CSC and not c.CTX_INIT:
            print("Initializing class-specific contexts")
        elif not c.CTX_INIT:
            print("Initializing a generic context")
        truncate = cfg.get("NATIVE", {}).get("TRUNCATE_PROMPTS", True)
        shared = cfg.get("NATIVE", {}).get("SHARED_PREFIX", True)
        ctx_vectors, self.prompt_prefix = init_prompts(
            self, classnames, clip_model, c.N_CTX, c.CTX_INIT, c.CLASS_TOKEN_POSITION,
            bool(c.CSC) and not c.CTX_INIT, truncate, shared, class_range)
        self.ctx = nn.Parameter(ctx_vectors)
        self.class_token_position = c.CLASS_TOKEN_POSITION

    def assemble(self):
        """Text-encoder input rows (prompts + positional embedding) of the classes this
        process encodes (all of them unless class-sharded), grad -> ctx."""
        lo, hi = self.class_range
        ctx = self.ctx[lo:hi] if (self.ctx.dim() == 3 and (lo, hi) != (0, self.n_cls)) else self.ctx
        return PromptAssembleFn.apply(ctx, None, self.layout)

    def forward(self):
        ctx = self.ctx
        if ctx.dim() == 2:
            ctx = ctx.unsqueeze(0).expand(self.n_cls, -1, -1)
        prefix, suffix = self.token_prefix, self.token_suffix
        if self.class_token_position == "end":
            return torch.cat([prefix, ctx, suffix], dim=1)
        rows = []
        for i in range(self.n_cls):
            nl = self.name_lens[i]
            cls_i, suf_i = suffix[i:i + 1, :nl], suffix[i:i + 1, nl:]
            if self.class_token_position == "middle":
                h = self.n_ctx // 2
                rows.append(torch.cat([prefix[i:i + 1], ctx[i:i + 1, :h], cls_i, ctx[i:i + 1, h:], suf_i], 1))
            elif self.class_token_position == "front":
                rows.append(torch.cat([prefix[i:i + 1], cls_i, ctx[i:i + 1], suf_i], 1))
            else:
                raise ValueError("Unknown class_token_position")
        return torch.cat(rows, dim=0)


class CustomCLIP(ImageFeatureSchedule, nn.Module):
    """coop.py:302-390. ``class_counts`` (per-rank class counts, rank order) turns on
    class-sharded text encoding: this process encodes only its classes and the [C, E] text
    features are all-gathered (dist.AllGatherRows: in backward the text-feature gradient
    is reduce-scattered back to the class owners). In eval mode without autograd the text
    features are computed once and reused until ctx changes (the reference re-encodes all
    C prompts on every test batch, coop.py:356-363)."""

    def __init__(self, cfg, classnames, clip_model, class_counts=None):
        super().__init__()
        self.cfg = cfg
        self.class_counts = class_counts
        class_range = None
        if class_counts is not None:
            lo = sum(class_counts[:dist.rank()])
            class_range = (lo, lo + class_counts[dist.rank()])
        self.prompt_learner = PromptLearner(cfg, classnames, clip_model, class_range)
        self.tokenized_prompts = self.prompt_learner.tokenized_prompts
        self.image_encoder = clip_model.visual
        self.text_encoder = TextEncoder(clip_model)
        self.text_core = clip_model.text
        self.logit_scale = clip_model.logit_scale
        self.logit_scale_value = clip_model.logit_scale_value
        self.dtype = clip_model.dtype
        self.loss_type = cfg.TRAINER.COOP.get("LOSS_TYPE", "ce")
        if self.loss_type == "simclr":
            print(">> Using LogitsNTXentLoss (logit-based simclr)!")
            self.criterion_simclr = LogitsNTXentLoss(temperature=0.07)
        elif self.loss_type == "ce":
            print(">> Using CE Loss!")
            self.criterion_ce = CrossEntropyLoss()
        elif self.loss_type == "focal":
            print(">> Use Focal Loss!")
            alpha = focal_alpha(cfg.DATASET.PER_CLASS_SHOTS, len(classnames), zero_guard=True)
            self.criterion_ce = MultiClassFocalLoss(alpha=alpha, gamma=2, reduction="mean")
        else:
            raise ValueError(f"Unknown loss_type = {self.loss_type}")

    def text_features(self):
        pl = self.prompt_learner
        x0 = pl.assemble()
        txt = TextEncodeFn.apply(x0, self.text_core, pl.layout.shape(1))
        if self.class_counts is not None:
            txt = dist.AllGatherRows.apply(txt, self.class_counts)
        return txt

    def _cached_text_features(self):
        ctx = self.prompt_learner.ctx
        key = (ctx.data_ptr(), ctx._version, getattr(ctx, "_clipk_gen", 0))
        cache = getattr(self, "_txt_cache", None)
        if cache is None or cache[0] != key:
            cache = self._txt_cache = (key, self.text_features())
        return cache[1]

    def train(self, mode=True):
        self._txt_cache = None
        return super().train(mode)

    def prepare_eval(self):
        """Called by TrainerX.test before its batch loop: encode (and, class-sharded,
        all-gather) the class prompts now, so every rank joins that collective exactly once
        -- a rank whose test shard is empty would otherwise never reach it and the others
        would wait forever."""
        if not self.training and not torch.is_grad_enabled():
            self._cached_text_features()

    def forward_once(self, image):
        """The image features come prefetched (NATIVE.PREFETCH_VISION), or from this step's
        first forward (the post-step accuracy forward of the same images), or -- NATIVE.
        OVERLAP_VISION -- from a side stream beside the image-independent text encoder
        (trainers/_vision.py); all bitwise the inline result."""
        imf = self.cached_image_features(image)
        join = None
        if imf is None:
            if (image.is_cuda and self.cfg.get("NATIVE", {}).get("OVERLAP_VISION", False)
                    and (self.training or torch.is_grad_enabled())):
                join = self.image_features_async(image)
            else:
                imf = self.image_features(image)
        if not self.training and not torch.is_grad_enabled():
            txt = self._cached_text_features()
        else:
            txt = self.text_features()
        if join is not None:
            imf = join()
        return CosineLogitsFn.apply(imf, txt, self.logit_scale_value, 0, self.prompt_learner.n_cls)

    def forward(self, img1, lbl=None, img2=None):
        if self.loss_type == "simclr":
            return self.criterion_simclr(self.forward_once(img1), self.forward_once(img2))
        if self.loss_type in ("ce", "focal"):
            logits = self.forward_once(img1)
            if self.training and lbl is not None:
                return self.criterion_ce(logits, lbl)
            return logits
        raise ValueError(f"Unsupported loss_type? {self.loss_type}")


@TRAINER_REGISTRY.register()
class CoOp(TrainerX):
    """coop.py:396-510 trainer contract: build_model / forward_backward / parse_batch_train /
    load_model. Multi-GPU: one process per GPU (see fsp_amd.dist), not nn.DataParallel."""

    def check_cfg(self, cfg):
        assert cfg.TRAINER.COOP.PREC in ["fp16", "fp32", "amp", "bf16", "fp32s"]

    def build_model(self):
        cfg = self.cfg
        classnames = self.dm.dataset.classnames
        clip_model = load_clip(cfg, cfg.TRAINER.COOP.PREC, self.device)
        print("Building custom CLIP w. logit-simclr or CE")
        counts = None
        if dist.world_size() > 1 and cfg.get("NATIVE", {}).get("CLASS_SHARD", True):
            w = dist.world_size()
            counts = [hi - lo for lo, hi in (dist.shard_range(len(classnames), r, w) for r in range(w))]
        self.model = CustomCLIP(cfg, classnames, clip_model, class_counts=counts)
        for name, param in self.model.named_parameters():
            if "prompt_learner" not in name:
                param.requires_grad = False
        if cfg.MODEL.INIT_WEIGHTS:
            self.load_pretrained_weights(self.model.prompt_learner, cfg.MODEL.INIT_WEIGHTS)
        self.optim = build_optimizer(self.model.prompt_learner, cfg.OPTIM)
        self.sched = build_lr_scheduler(self.optim, cfg.OPTIM)
        self.register_model("prompt_learner", self.model.prompt_learner, self.optim, self.sched)

    def forward_backward(self, batch):
        """coop.py:438-474. Multi-GPU: the loss is scaled by this rank's share of the global
        batch before backward and the prompt gradients all-reduced (TrainerX). PREC amp: the
        step is skipped when a gradient is not finite, as GradScaler.step does (the bf16
        backward needs no loss scaling)."""
        x1, lbl, x2 = self.parse_batch_train(batch)
        nb, self.next_batch = getattr(self, "next_batch", None), None
        if (nb is not None and x1.is_cuda and x2 is None
                and self.cfg.get("NATIVE", {}).get("PREFETCH_VISION", False)):
            # the next step's image features on a side stream for the whole of this step
            # (run_epoch / bench set next_batch; trainers/_vision.py)
            self.model.prefetch_image_features(self.parse_batch_train(nb)[0])
        loss = self.model(x1, lbl, x2)
        self.optim.zero_grad()
        w = self.batch_weight(batch, x1.shape[0])
        (loss * w if w != 1.0 else loss).backward()
        self.allreduce_grads(self.model.prompt_learner)
        if self.cfg.TRAINER.COOP.PREC != "amp" or grads_finite(self.model.prompt_learner):
            self.optim.step()
        loss_summary = LossSummary()
        loss_summary["loss"] = loss
        if lbl is not None and x2 is None and self.model.loss_type == "ce":
            # coop.py:464-469: acc from a second forward AFTER the step
            with torch.no_grad():
                logits_eval = self.model(x1, lbl=None, img2=None)
                loss_summary["acc"] = compute_accuracy(logits_eval, lbl)[0]
        if (self.batch_idx + 1) == self.num_batches:
            self.update_lr()
        return loss_summary

    def parse_batch_train(self, batch):
        if self.cfg.TRAINER.COOP.LOSS_TYPE == "simclr":
            return batch["img1"].to(self.device), None, batch["img2"].to(self.device)
        return batch["img"].to(self.device), batch["label"].to(self.device), None

    def load_model(self, directory, epoch=None):
        if not directory:
            print("no pretrained => skip")
            return
        model_file = "model-best.pth.tar" if not epoch else f"model.pth.tar-{epoch}"
        for name in self.get_model_names():
            model_path = osp.join(directory, name, model_file)
            if not osp.exists(model_path):
                raise FileNotFoundError(f"No model at {model_path}")
            ckpt = self.load_checkpoint(model_path)
            state_dict = ckpt["state_dict"]
            state_dict.pop("token_prefix", None)
            state_dict.pop("token_suffix", None)
            print(f'Loading {name} from "{model_path}" (epoch={ckpt["epoch"]})')
            self._models[name].load_state_dict(state_dict, strict=False)
