"""Losses of the fork (PromptSRC/trainers/coop.py:66-163, cocoop.py:66-101).

CE and the class-frequency-weighted focal loss run as one fused HIP kernel (forward
and dlogits together, ``clipk_ce_loss``). The logit-space NT-Xent loss (CoOp
LOSS_TYPE "simclr") operates on the tiny [2B, 2B] similarity of L2-normalised logits
and is composed from torch ops (vectorised form of the reference's per-row loop).
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from ._fns import CrossEntropyFn


class CrossEntropyLoss(nn.Module):
    def forward(self, logits, targets):
        return CrossEntropyFn.apply(logits, targets, None, 0.0, False)


class MultiClassFocalLoss(nn.Module):
    def __init__(self, alpha=None, gamma=2, reduction="mean"):
        super().__init__()
        if isinstance(alpha, list):
            self.alpha = torch.tensor(alpha, dtype=torch.float32)
        elif isinstance(alpha, torch.Tensor):
            self.alpha = alpha.float()
        elif alpha is None:
            self.alpha = None
        else:
            raise TypeError("alpha must be None, list, or torch.Tensor")
        self.gamma = float(gamma)
        self.reduction = reduction

    def forward(self, inputs, targets):
        a = None
        if self.alpha is not None:
            if self.alpha.device != inputs.device:
                self.alpha = self.alpha.to(inputs.device)
            a = self.alpha
        # reduction: 'mean' / 'sum', anything else returns the per-sample losses (coop.py:158-163)
        red = self.reduction if self.reduction in ("mean", "sum") else "none"
        return CrossEntropyFn.apply(inputs, targets, a, self.gamma, True, red)


class LogitsNTXentLoss(nn.Module):
    def __init__(self, temperature=0.07):
        super().__init__()
        self.temperature = temperature

    def forward(self, logits1, logits2):
        z = torch.cat([F.normalize(logits1, dim=1), F.normalize(logits2, dim=1)], 0)
        n2 = z.shape[0]
        n = n2 // 2
        sim = z @ z.t() / self.temperature
        idx = torch.arange(n2, device=z.device)
        pos = torch.cat([idx[:n] + n, idx[n:] - n])
        keep = (idx[None, :] != idx[:, None]) & (idx[None, :] != pos[:, None])
        neg = sim[keep].view(n2, n2 - 2)
        out = torch.cat([sim[idx, pos][:, None], neg], 1)
        return F.cross_entropy(out, torch.zeros(n2, dtype=torch.long, device=z.device))


def focal_alpha(per_class, n_cls, zero_guard):
    """alpha_c = total / (C * n_c) (coop.py:336-346 with the zero guard; cocoop.py:221-230
    without it, where a zero count raises ZeroDivisionError as in the reference)."""
    if per_class is None or (isinstance(per_class, (list, tuple)) and len(per_class) == 0):
        return None
    if isinstance(per_class, str):
        per_class = list(map(int, per_class.strip("[]").split(",")))
    total = sum(per_class)
    if zero_guard:
        return [total / (n_cls * c) if c > 0 else 0.0 for c in per_class]
    return [total / (n_cls * c) for c in per_class]
