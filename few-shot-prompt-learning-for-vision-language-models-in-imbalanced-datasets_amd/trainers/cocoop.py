"""CoCoOp on the MI355X-native path — same registry name, cfg keys (TRAINER.COCOOP.*),
module contract and checkpoint format as ``PromptSRC/trainers/cocoop.py``.

The reference encodes the C class prompts once PER IMAGE in a Python loop
(cocoop.py:247-251) after materialising [B, C, 77, W] prompts (cocoop.py:189-197).
Here one launch sequence encodes all B*C conditional prompts at once: the Meta-Net
bias is added inside the prompt-assembly kernel, the text encoder runs over
B*C sequences truncated to L = max EOT + 1, and the per-image cosine logits come from
one kernel. Large B*C is split into image chunks bounded by NATIVE.MAX_TEXT_ROWS.

Multi-GPU (one process per GPU, ``NATIVE.COCOOP_SHARD``):
* "image" (default): data parallel over images -- each rank encodes its images' B_r*C
  prompts, one averaged all-reduce of the ctx + Meta-Net gradients;
* "class" (SURVEY §8(e) Option B, for the reference's batch-1 configs,
  configs/trainers/CoCoOp/vit_b16_c4_ep10_batch1_ctxv1.yaml:3): every rank scores the SAME
  batch against its C/W classes (shard_range), the [B, C_r] logit slices are all-gathered
  (dist.GatherClassColumns), every rank evaluates the full loss and back-propagates its own
  classes, and the partial prompt gradients are SUM all-reduced. The global batch (and so
  the update) is the single-process one at any world size.
"""
from __future__ import annotations

import os.path as osp
from collections import OrderedDict

import torch
import torch.nn as nn

from .. import dist
from ..engine.registry import TRAINER_REGISTRY
from ..engine.trainer import TrainerX, load_clip
from ..engine.optim import build_optimizer, build_lr_scheduler
from ..engine.metrics import LossSummary
from ..clip.model import TextEncodeFn
from ._fns import PromptAssembleFn, CosineLogitsFn, MetaNetFn, MetaNetNormFn, backward_unit
from .losses import CrossEntropyLoss, MultiClassFocalLoss, focal_alpha
from ._vision import ImageFeatureSchedule
from .prompt_base import init_prompts, grads_finite
from .coop import TextEncoder  # noqa: F401  (same API-compatible text encoder)


class MetaNet(nn.Module):
    """nn.Sequential(linear1, relu, linear2) of cocoop.py:139-143 (same state-dict keys)."""

    def __init__(self, vis_dim, ctx_dim):
        super().__init__()
        self.linear1 = nn.Linear(vis_dim, vis_dim // 16)
        self.linear2 = nn.Linear(vis_dim // 16, ctx_dim)

    def forward(self, x):
        return MetaNetFn.apply(x, self.linear1.weight, self.linear1.bias, self.linear2.weight,
                               self.linear2.bias)

    def forward_normalized(self, x):
        """(meta_net(x / |x|), x / |x|) in one launch (MetaNetNormFn)."""
        return MetaNetNormFn.apply(x, self.linear1.weight, self.linear1.bias, self.linear2.weight,
                                   self.linear2.bias)


class PromptLearner(nn.Module):
    def __init__(self, cfg, classnames, clip_model, class_range=None):
        super().__init__()
        c = cfg.TRAINER.COCOOP
        clip_imsize = clip_model.visual.input_resolution
        cfg_imsize = cfg.INPUT.SIZE[0]
        assert cfg_imsize == clip_imsize, f"cfg_imsize({cfg_imsize}) != clip_imsize({clip_imsize})"
        vis_dim = clip_model.visual.output_dim
        ctx_dim = clip_model.arch.transformer_width
        truncate = cfg.get("NATIVE", {}).get("TRUNCATE_PROMPTS", True)
        shared = cfg.get("NATIVE", {}).get("SHARED_PREFIX", True)
        ctx_vectors, self.prompt_prefix = init_prompts(self, classnames, clip_model, c.N_CTX, c.CTX_INIT,
                                                       "end", False, truncate, shared, class_range)
        self.ctx = nn.Parameter(ctx_vectors)
        self.meta_net = MetaNet(vis_dim, ctx_dim).to(ctx_vectors.device)

    def assemble(self, im_features):
        """im_features [B, V] (L2-normalised) -> x0 [B*C*L, W] with ctx + meta_net(imf_b)."""
        bias = self.meta_net(im_features)
        return PromptAssembleFn.apply(self.ctx, bias, self.layout)

    def assemble_raw(self, im_features):
        """im_features [B, V] as the image encoder returns them -> (x0, imf / |imf|): the
        normalisation of cocoop.py:238 inside the Meta-Net launch."""
        bias, imf_n = self.meta_net.forward_normalized(im_features)
        return PromptAssembleFn.apply(self.ctx, bias, self.layout), imf_n

    def construct_prompts(self, ctx, prefix, suffix, label=None):
        if label is not None:
            prefix, suffix = prefix[label], suffix[label]
        return torch.cat([prefix, ctx, suffix], dim=1)

    def forward(self, im_features):
        """API-compatible [B, C, 77, W] prompts (cocoop.py:173-198)."""
        bias = self.meta_net(im_features).unsqueeze(1)
        shifted = self.ctx.unsqueeze(0) + bias
        out = [self.construct_prompts(s.unsqueeze(0).expand(self.n_cls, -1, -1), self.token_prefix,
                                      self.token_suffix) for s in shifted]
        return torch.stack(out, 0)


class CustomCLIP(ImageFeatureSchedule, nn.Module):
    """cocoop.py:200-260. ``class_counts`` (per-rank class counts, rank order) turns on class
    sharding: this process encodes its classes for every image and the logit slices are
    all-gathered (module doc)."""

    def __init__(self, cfg, classnames, clip_model, class_counts=None):
        super().__init__()
        self.cfg = cfg
        self.class_counts = class_counts
        class_range = None
        if class_counts is not None:
            if min(class_counts) < 1:
                raise ValueError(f"class sharding needs >= 1 class per rank, got counts {class_counts}")
            lo = sum(class_counts[:dist.rank()])
            class_range = (lo, lo + class_counts[dist.rank()])
        self.prompt_learner = PromptLearner(cfg, classnames, clip_model, class_range)
        self.tokenized_prompts = self.prompt_learner.tokenized_prompts
        self.image_encoder = clip_model.visual
        self.text_core = clip_model.text
        self.text_encoder = TextEncoder(clip_model)
        self.logit_scale = clip_model.logit_scale
        self.logit_scale_value = clip_model.logit_scale_value
        self.dtype = clip_model.dtype
        self.max_rows = int(cfg.get("NATIVE", {}).get("MAX_TEXT_ROWS", 2_000_000))
        # class-sharded: every rank must split a batch into the same number of logits_for calls
        # (each runs a GatherClassColumns collective), so the chunking uses the largest rank's
        # text rows per image (one MAX all-reduce here, at construction on every rank)
        self._rows_per_img = self.prompt_learner.layout.rows_per_group
        if class_counts is not None:
            self._rows_per_img = int(dist.max_over_ranks(float(self._rows_per_img)))
        self.use_focal_loss = cfg.TRAINER.COCOOP.get("USE_FOCAL_LOSS", False)
        print(f">> USE_FOCAL_LOSS = {self.use_focal_loss}")
        if self.use_focal_loss:
            print(">> Use Focal Loss!")
            per_class = getattr(cfg.DATASET, "PER_CLASS_SHOTS", None)
            alpha = focal_alpha(per_class, len(classnames), zero_guard=False) \
                if isinstance(per_class, (list, str)) else None
            self.criterion = MultiClassFocalLoss(alpha=alpha, gamma=2, reduction="mean")
        else:
            print(">> Use Cross Entropy Loss!")
            self.criterion = CrossEntropyLoss()

    def logits_for(self, imf):
        """imf: the raw image features (normalised with the Meta-Net, assemble_raw)."""
        pl = self.prompt_learner
        B = imf.shape[0]
        x0, imf_n = pl.assemble_raw(imf)
        txt = TextEncodeFn.apply(x0, self.text_core, pl.layout.shape(B))
        logits = CosineLogitsFn.apply(imf_n, txt, self.logit_scale_value, 1, pl.layout.n_cls)
        if self.class_counts is not None:
            logits = dist.GatherClassColumns.apply(logits, self.class_counts)
        return logits

    def forward(self, image, label=None):
        imf = self.image_features(image)
        nxt, self.next_image = getattr(self, "next_image", None), None
        if nxt is not None and not self.training and self.cfg.get("NATIVE", {}).get("PREFETCH_VISION", False):
            # eval: the next test batch's image encoder beside this batch's text encoder (the test
            # loop names it, TrainerX.test)
            self.prefetch_image_features(nxt)
        # imf / imf.norm(dim=-1, keepdim=True) (cocoop.py:238) happens in logits_for's Meta-Net launch
        pl = self.prompt_learner
        chunk = max(1, self.max_rows // self._rows_per_img)
        if imf.shape[0] <= chunk:
            logits = self.logits_for(imf)
        else:
            logits = torch.cat([self.logits_for(imf[i:i + chunk]) for i in range(0, imf.shape[0], chunk)], 0)
        if self.training and label is not None:
            return self.criterion(logits, label)
        return logits


@TRAINER_REGISTRY.register()
class CoCoOp(TrainerX):
    """cocoop.py:262-370 trainer contract."""

    def check_cfg(self, cfg):
        assert cfg.TRAINER.COCOOP.PREC in ["fp16", "fp32", "amp", "bf16", "fp32s"]
        mode = cfg.get("NATIVE", {}).get("COCOOP_SHARD", "image")
        if mode not in ("image", "class"):
            raise ValueError(f"NATIVE.COCOOP_SHARD must be 'image' or 'class', got {mode!r}")

    @property
    def class_sharded(self) -> bool:
        return dist.batches_replicated(self.cfg)

    def build_model(self):
        cfg = self.cfg
        classnames = self.dm.dataset.classnames
        print(f"Loading CLIP (backbone: {cfg.MODEL.BACKBONE.NAME})")
        clip_model = load_clip(cfg, cfg.TRAINER.COCOOP.PREC, self.device)
        print("Building custom CLIP")
        counts = None
        if self.class_sharded:
            w = dist.world_size()
            counts = [hi - lo for lo, hi in (dist.shard_range(len(classnames), r, w) for r in range(w))]
        self.model = CustomCLIP(cfg, classnames, clip_model, class_counts=counts)
        print("Turning off gradients in both the image and the text encoder")
        for name, param in self.model.named_parameters():
            if "prompt_learner" not in name:
                param.requires_grad_(False)
        enabled = {n for n, p in self.model.named_parameters() if p.requires_grad}
        print(f"Parameters to be updated: {enabled}")
        if cfg.MODEL.INIT_WEIGHTS:
            self.load_pretrained_weights(self.model.prompt_learner, cfg.MODEL.INIT_WEIGHTS)
        self.optim = build_optimizer(self.model.prompt_learner, cfg.OPTIM)
        self.sched = build_lr_scheduler(self.optim, cfg.OPTIM)
        self.register_model("prompt_learner", self.model.prompt_learner, self.optim, self.sched)

    def forward_backward(self, batch):
        """cocoop.py:313-338 (multi-GPU weighting and the amp skip test as CoOp's).
        PREC fp32s, one process: the text backward's overflow flag (a retry at a lower gradient
        scale, TextEncoderCore.backward) is not waited for inside the step. The SGD launch skips
        itself on the device when the flag is set, and the flag of step i is read in step i + 1
        once its forward is queued (the GPU is busy meanwhile): an overflowed step i is then re-run
        at the lower scale and step i + 1's forward again -- the same updates as the waiting form
        (0.6 ms/step of host synchronisation at B = 8, 0.3 at B = 1: tools/lab/step_parts.py)."""
        image, label = self.parse_batch_train(batch)
        nb, self.next_batch = getattr(self, "next_batch", None), None
        nxt = ready = None
        if nb is not None and image.is_cuda and self.cfg.get("NATIVE", {}).get("PREFETCH_VISION", False):
            # the next step's image features on a side stream beside this step (run_epoch /
            # bench set next_batch to the batch the loop will pass next; trainers/_vision.py),
            # from this point of the main stream on
            nxt = self.parse_batch_train(nb)[0]
            ready = torch.cuda.Event()
            ready.record(torch.cuda.current_stream(image.device))
        defer = self._deferred_status()
        loss = self.model(image, label)
        if nxt is not None:
            # issued after this step's forward, so that the host queues the main stream's work
            # first after a synchronisation
            self.model.prefetch_image_features(nxt, after=ready)
        if self._settle_pending():
            loss = self.model(image, label)  # the re-run step before changed the prompts
        return self._finish_step(batch, image, loss, defer)

    def _finish_step(self, batch, image, loss, defer, redo=False):
        """Backward, gradient all-reduce, SGD and the LR update of forward_backward; defer: the
        split status whose check is left to the next step (None: checked in the backward)."""
        self.optim.zero_grad()
        if self.class_sharded:  # full loss on every rank, partial gradients: summed
            backward_unit(loss)
            dist.allreduce_grads([p for p in self.model.prompt_learner.parameters() if p.requires_grad],
                                 average=False)
        else:
            w = self.batch_weight(batch, image.shape[0])
            if w != 1.0:
                (loss * w).backward()
            else:
                backward_unit(loss)  # loss.backward() without the seed fill / multiply launches
            self.allreduce_grads(self.model.prompt_learner)
        lrs = [g["lr"] for g in self.optim.param_groups]
        if self.cfg.TRAINER.COCOOP.PREC != "amp" or grads_finite(self.model.prompt_learner):
            if defer is not None:
                self.optim.step(guard=(defer.flags, 2))  # skipped on the device after an overflow
                self._pending = (defer.take_async(), batch, lrs, getattr(self.optim, "created_last", []))
            else:
                self.optim.step()
        loss_summary = LossSummary()
        loss_summary["loss"] = loss
        if not redo and (self.batch_idx + 1) == self.num_batches:
            self.update_lr()
        return loss_summary

    def _deferred_status(self):
        """The text encoder's split status when its check may be deferred (PREC fp32s, one
        process, NATIVE.DEFER_SPLIT_CHECK), else None (the backward checks it itself)."""
        core = self.model.text_core
        st = getattr(core, "_status", None)
        on = (st is not None and not dist.is_dist() and self.cfg.get("NATIVE", {}).get("DEFER_SPLIT_CHECK", True)
              and hasattr(self.optim, "created_last"))
        core.defer_check = bool(on)
        return st if on else None

    def _settle_pending(self):
        """Read the previous step's deferred overflow flag (waits for that step only). On an
        overflow -- its SGD was skipped on the device -- re-run that step with the check in the
        backward (lower-scale retry), at its own LR. Returns whether a step was re-run."""
        pend, self._pending = getattr(self, "_pending", None), None
        if pend is None:
            return False
        handle, batch, lrs, created = pend
        if not handle.result() & 2:
            return False
        torch.cuda.synchronize()
        for p in created:  # momentum buffers the skipped step created: never written
            self.optim.state.pop(p, None)
        now = [g["lr"] for g in self.optim.param_groups]
        core = self.model.text_core
        was = core.defer_check
        try:
            for g, lr in zip(self.optim.param_groups, lrs):
                g["lr"] = lr
            core.defer_check = False
            image, label = self.parse_batch_train(batch)
            self._finish_step(batch, image, self.model(image, label), None, redo=True)
        finally:
            for g, lr in zip(self.optim.param_groups, now):
                g["lr"] = lr
            core.defer_check = was  # (this step's own backward defers again)
        type(self).deferred_redos += 1
        return True

    deferred_redos = 0  # steps re-run after a deferred overflow check, all instances

    def flush_deferred(self):
        """Settle the last step's deferred check (end of an epoch, before a test or a save)."""
        with torch.enable_grad():  # (test() runs under no_grad; a re-run step needs autograd)
            self._settle_pending()

    def parse_batch_train(self, batch):
        return batch["img"].to(self.device), batch["label"].to(self.device)

    def load_model(self, directory, epoch=None):
        if not directory:
            print("Note that load_model() is skipped as no pretrained model is given")
            return
        model_file = "model-best.pth.tar" if epoch is None else f"model.pth.tar-{epoch}"
        for name in self.get_model_names():
            model_path = osp.join(directory, name, model_file)
            if not osp.exists(model_path):
                raise FileNotFoundError(f'Model not found at "{model_path}"')
            checkpoint = self.load_checkpoint(model_path)
            state_dict = checkpoint["state_dict"]
            state_dict.pop("token_prefix", None)
            state_dict.pop("token_suffix", None)
            print(f'Loading weights to {name} from "{model_path}" (epoch = {checkpoint["epoch"]})')
            self._models[name].load_state_dict(state_dict, strict=False)
