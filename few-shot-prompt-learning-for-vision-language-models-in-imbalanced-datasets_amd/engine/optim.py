"""Optimizer + LR schedule for the prompt parameters.

``FusedSGD``: torch.optim.SGD semantics as Dassl builds it for CoOp/CoCoOp
(Dassl.pytorch/dassl/optim/optimizer.py:105-113: momentum 0.9, weight decay 5e-4,
dampening 0, no nesterov) with the update running in the clipk_sgd_step HIP kernel.
``WarmupCosineLR``: Dassl's ConstantWarmupScheduler(CosineAnnealingLR) per-epoch LR
(lr_scheduler.py:35-54,120-152); closed form, pinned by tests/golden/lr_schedule.npz.
"""
from __future__ import annotations

import math
import warnings

import torch

from .. import ops


class FusedSGD(torch.optim.Optimizer):
    """Param groups carry every key of torch.optim.SGD's groups, so ``state_dict()`` loads
    into the reference's torch.optim.SGD (and a reference SGD state into this one)."""

    created_last = ()

    def __init__(self, params, lr=0.002, momentum=0.9, weight_decay=5e-4, dampening=0.0,
                 nesterov=False):
        if dampening != 0 or nesterov:
            raise ValueError("FusedSGD implements dampening=0, nesterov=False (the Dassl CoOp setup)")
        super().__init__(params, dict(lr=lr, momentum=momentum, dampening=0, weight_decay=weight_decay,
                                      nesterov=False, maximize=False, foreach=None, differentiable=False,
                                      fused=None))

    @staticmethod
    def defer_grad_scale(grads, s):
        """The next step updates with s * g for these gradient tensors (dist.allreduce_grads folds
        the average of a SUM all-reduce here: one launch less per step). A tag on each tensor,
        set (not multiplied) per all-reduce and consumed by step()."""
        for g in grads:
            g._clipk_grad_scale = s

    @torch.no_grad()
    def step(self, closure=None, guard=None):
        """guard = (int32 device flags, mask): the update is skipped on the device when
        flags[0] & mask (clipk_sgd_step_multi_if); ``created_last`` lists the parameters whose
        momentum buffer this call created (a skipped step's are never written)."""
        loss = closure() if closure is not None else None
        self.created_last = []
        for grp in self.param_groups:
            # the group's tensors in one launch per 16 (clipk_sgd_step_multi): at the reference's
            # batch of 1 the five per-tensor launches were kernel boundaries on the critical path
            ps, gs, bufs, has, scales = [], [], [], [], []
            for p in grp["params"]:
                if p.grad is None:
                    continue
                if not p.is_cuda:
                    raise RuntimeError("FusedSGD runs on the GPU only (HIP kernel); no CPU path")
                if grp.get("dampening", 0) != 0 or grp.get("nesterov", False) or grp.get("maximize", False):
                    raise ValueError("FusedSGD implements dampening=0, nesterov=False, maximize=False")
                if p.dtype != torch.float32 or not p.is_contiguous():
                    raise ValueError("FusedSGD: fp32 contiguous parameters")
                st = self.state[p]
                buf = st.get("momentum_buffer")
                h = buf is not None
                if not h:
                    buf = st["momentum_buffer"] = torch.empty_like(p)
                    self.created_last.append(p)
                elif buf.device != p.device or not buf.is_contiguous():
                    buf = st["momentum_buffer"] = buf.to(p.device).contiguous()
                ps.append(p.data)
                scales.append(getattr(p.grad, "_clipk_grad_scale", 1.0))
                if hasattr(p.grad, "_clipk_grad_scale"):
                    del p.grad._clipk_grad_scale
                gs.append(p.grad if p.grad.is_contiguous() else p.grad.contiguous())
                bufs.append(buf)
                has.append(h)
                p._clipk_gen = getattr(p, "_clipk_gen", 0) + 1  # invalidates cached text features
            if ps:
                if len(set(scales)) > 1:  # (mixed tags: scaled here, then one unscaled launch)
                    gs = [g * sc if sc != 1.0 else g for g, sc in zip(gs, scales)]
                    scales = [1.0]
                ops.sgd_step_multi(ps, gs, bufs, grp["lr"], grp["momentum"], grp["weight_decay"], has,
                                   grad_scale=scales[0], guard=guard)
        return loss


def warmup_cosine_lr(epoch: int, base_lr: float, max_epoch: int, warmup_epoch: int = -1,
                     warmup_type: str = "constant", warmup_cons_lr: float = 1e-5,
                     warmup_min_lr: float = 1e-5, warmup_recount: bool = True) -> float:
    if warmup_epoch > 0 and epoch < warmup_epoch:
        if warmup_type == "constant":
            return warmup_cons_lr
        if warmup_type == "linear":  # LinearWarmupScheduler
            return epoch / warmup_epoch * base_lr if epoch > 0 else warmup_min_lr
        raise ValueError(warmup_type)
    # the cosine successor restarts its count after warmup unless WARMUP_RECOUNT is off
    # (lr_scheduler.py:128-130: then it starts at last_epoch = WARMUP_EPOCH)
    e = epoch - warmup_epoch if (warmup_epoch > 0 and warmup_recount) else epoch
    return 0.5 * base_lr * (1 + math.cos(math.pi * e / max_epoch))


class WarmupCosineLR:
    """Epoch-stepped scheduler with the Dassl get_last_lr()/step()/state_dict() surface.

    ``state_dict()`` has the shape of the scheduler Dassl's build_lr_scheduler returns
    (lr_scheduler.py:128-152): with warmup, the __dict__ of a Constant/LinearWarmupScheduler
    including its ``successor`` -- a torch CosineAnnealingLR advanced to the same epoch (on a
    detached one-parameter SGD, as a resumed Dassl successor is) -- so the reference's
    ``resume_from_checkpoint`` restores it; without warmup, a CosineAnnealingLR state dict.
    ``load_state_dict`` needs only ``last_epoch`` (the LR is a closed form of it)."""

    def __init__(self, optimizer, optim_cfg):
        self.opt = optimizer
        self.cfg = optim_cfg
        self.base_lr = optim_cfg.LR
        self.last_epoch = 0
        for g in self.opt.param_groups:
            g.setdefault("initial_lr", g["lr"])
        self._apply()

    def _lr(self, e):
        c = self.cfg
        return warmup_cosine_lr(e, c.LR, c.MAX_EPOCH, c.WARMUP_EPOCH, c.WARMUP_TYPE, c.WARMUP_CONS_LR,
                                c.WARMUP_MIN_LR, c.get("WARMUP_RECOUNT", True))

    def _apply(self):
        for g in self.opt.param_groups:
            g["lr"] = self._lr(self.last_epoch)

    def step(self):
        self.last_epoch += 1
        self._apply()

    def get_last_lr(self):
        return [g["lr"] for g in self.opt.param_groups]

    def _cosine_state(self, epochs):
        c = self.cfg
        return {"T_max": float(c.MAX_EPOCH), "eta_min": 0.0, "base_lrs": [c.LR] * len(self.opt.param_groups),
                "last_epoch": epochs, "_step_count": epochs + 1,
                "_get_lr_called_within_step": False, "_is_initial": False,
                "_last_lr": [0.5 * c.LR * (1 + math.cos(math.pi * epochs / c.MAX_EPOCH))] * len(self.opt.param_groups)}

    def state_dict(self):
        c = self.cfg
        n = len(self.opt.param_groups)
        if not (c.WARMUP_EPOCH > 0):
            return self._cosine_state(self.last_epoch)
        # the successor: stepped only after the warmup epochs (lr_scheduler.py:27-33)
        done = max(0, self.last_epoch - c.WARMUP_EPOCH)
        start = 0 if c.get("WARMUP_RECOUNT", True) else c.WARMUP_EPOCH
        dummy = torch.optim.SGD([torch.nn.Parameter(torch.zeros(1))], lr=c.LR)
        succ = torch.optim.lr_scheduler.CosineAnnealingLR(dummy, float(c.MAX_EPOCH))
        succ.last_epoch = start
        with warnings.catch_warnings():  # the detached optimizer never steps
            warnings.simplefilter("ignore")
            for _ in range(done):
                succ.step()
        # Dassl's warmup wrapper stops counting once the successor takes over (its step()
        # only steps the successor past warmup, lr_scheduler.py:27-33)
        outer = min(self.last_epoch, c.WARMUP_EPOCH)
        sd = {"successor": succ, "warmup_epoch": c.WARMUP_EPOCH, "base_lrs": [c.LR] * n,
              "last_epoch": outer, "_step_count": outer + 1,
              "_get_lr_called_within_step": False, "_is_initial": False,
              "_last_lr": [g["lr"] for g in self.opt.param_groups]}
        if c.WARMUP_TYPE == "constant":
            sd["cons_lr"] = c.WARMUP_CONS_LR
        else:
            sd["min_lr"] = c.WARMUP_MIN_LR
        return sd

    def load_state_dict(self, sd):
        """Epochs stepped so far, from our state or a Dassl one: past warmup, Dassl keeps the
        wrapper's last_epoch at WARMUP_EPOCH and counts on in the successor (whose count
        starts at 0, or at WARMUP_EPOCH without WARMUP_RECOUNT)."""
        c = self.cfg
        e = int(sd["last_epoch"])
        succ = sd.get("successor")
        if c.WARMUP_EPOCH > 0 and e >= c.WARMUP_EPOCH:
            s_last = getattr(succ, "last_epoch", None) if not isinstance(succ, dict) else succ.get("last_epoch")
            if s_last is not None:
                start = 0 if c.get("WARMUP_RECOUNT", True) else c.WARMUP_EPOCH
                e = c.WARMUP_EPOCH + int(s_last) - start
        self.last_epoch = e
        self._apply()


def build_optimizer(module, optim_cfg):
    if optim_cfg.NAME != "sgd":
        raise NotImplementedError(f"Optimizer {optim_cfg.NAME} not implemented on this path")
    params = [p for p in module.parameters() if p.requires_grad]
    return FusedSGD(params, lr=optim_cfg.LR, momentum=optim_cfg.MOMENTUM,
                    weight_decay=optim_cfg.WEIGHT_DECAY, dampening=optim_cfg.SGD_DAMPNING,
                    nesterov=optim_cfg.SGD_NESTEROV)


def build_lr_scheduler(optimizer, optim_cfg):
    if optim_cfg.LR_SCHEDULER != "cosine":
        raise NotImplementedError(optim_cfg.LR_SCHEDULER)
    return WarmupCosineLR(optimizer, optim_cfg)
