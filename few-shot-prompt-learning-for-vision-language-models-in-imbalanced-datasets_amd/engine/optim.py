"""Optimizer + LR schedule for the prompt parameters.

``FusedSGD``: torch.optim.SGD semantics as Dassl builds it for CoOp/CoCoOp
(Dassl.pytorch/dassl/optim/optimizer.py:105-113: momentum 0.9, weight decay 5e-4,
dampening 0, no nesterov) with the update running in the clipk_sgd_step HIP kernel.
``WarmupCosineLR``: Dassl's ConstantWarmupScheduler(CosineAnnealingLR) per-epoch LR
(lr_scheduler.py:35-54,120-152); closed form, pinned by tests/golden/lr_schedule.npz.
"""
from __future__ import annotations

import math

import torch

from .. import ops


class FusedSGD(torch.optim.Optimizer):
    def __init__(self, params, lr=0.002, momentum=0.9, weight_decay=5e-4, dampening=0.0,
                 nesterov=False):
        if dampening != 0 or nesterov:
            raise ValueError("FusedSGD implements dampening=0, nesterov=False (the Dassl CoOp setup)")
        super().__init__(params, dict(lr=lr, momentum=momentum, weight_decay=weight_decay))

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        for grp in self.param_groups:
            for p in grp["params"]:
                if p.grad is None:
                    continue
                if not p.is_cuda:
                    raise RuntimeError("FusedSGD runs on the GPU only (HIP kernel); no CPU path")
                st = self.state[p]
                has = "momentum_buffer" in st
                if not has:
                    st["momentum_buffer"] = torch.empty_like(p)
                ops.sgd_step(p.data, p.grad.contiguous(), st["momentum_buffer"], grp["lr"], grp["momentum"],
                             grp["weight_decay"], has)
        return loss


def warmup_cosine_lr(epoch: int, base_lr: float, max_epoch: int, warmup_epoch: int = -1,
                     warmup_type: str = "constant", warmup_cons_lr: float = 1e-5,
                     warmup_min_lr: float = 1e-5) -> float:
    if warmup_epoch > 0 and epoch < warmup_epoch:
        if warmup_type == "constant":
            return warmup_cons_lr
        if warmup_type == "linear":  # LinearWarmupScheduler
            return epoch / warmup_epoch * base_lr if epoch > 0 else warmup_min_lr
        raise ValueError(warmup_type)
    e = epoch - warmup_epoch if warmup_epoch > 0 else epoch
    return 0.5 * base_lr * (1 + math.cos(math.pi * e / max_epoch))


class WarmupCosineLR:
    """Epoch-stepped scheduler with the Dassl get_last_lr()/step()/state_dict() surface."""

    def __init__(self, optimizer, optim_cfg):
        self.opt = optimizer
        self.cfg = optim_cfg
        self.base_lr = optim_cfg.LR
        self.last_epoch = 0
        self._apply()

    def _lr(self, e):
        c = self.cfg
        return warmup_cosine_lr(e, c.LR, c.MAX_EPOCH, c.WARMUP_EPOCH, c.WARMUP_TYPE, c.WARMUP_CONS_LR,
                                c.WARMUP_MIN_LR)

    def _apply(self):
        for g in self.opt.param_groups:
            g["lr"] = self._lr(self.last_epoch)

    def step(self):
        self.last_epoch += 1
        self._apply()

    def get_last_lr(self):
        return [g["lr"] for g in self.opt.param_groups]

    def state_dict(self):
        return {"last_epoch": self.last_epoch}

    def load_state_dict(self, sd):
        self.last_epoch = sd["last_epoch"]
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
