"""compute_accuracy (Dassl.pytorch/dassl/metrics/accuracy.py) and the Classification
evaluator (dassl/evaluation/evaluator.py:26-125): accuracy, error, macro-F1, per-class
accuracy. Predictions stay on the device until evaluate() (one host sync per eval,
instead of the reference's .item()/.cpu() per batch)."""
from __future__ import annotations

import numpy as np
import torch


def compute_accuracy(output, target, topk=(1,)):
    maxk = max(topk)
    batch_size = target.size(0)
    if isinstance(output, (tuple, list)):
        output = output[0]
    _, pred = output.topk(maxk, 1, True, True)
    pred = pred.t()
    correct = pred.eq(target.view(1, -1).expand_as(pred))
    res = []
    for k in topk:
        correct_k = correct[:k].reshape(-1).float().sum(0, keepdim=True)
        res.append(correct_k.mul_(100.0 / batch_size))
    return res


def macro_f1(y_true, y_pred):
    """sklearn f1_score(average='macro', labels=np.unique(y_true)), as Dassl's evaluator
    calls it (evaluator.py:71-76): classes only predicted, never present in y_true, are not
    averaged in."""
    labels = np.unique(y_true)
    f1s = []
    for c in labels:
        tp = np.sum((y_pred == c) & (y_true == c))
        fp = np.sum((y_pred == c) & (y_true != c))
        fn = np.sum((y_pred != c) & (y_true == c))
        denom = 2 * tp + fp + fn
        f1s.append(0.0 if denom == 0 else 2 * tp / denom)
    return float(np.mean(f1s)) if f1s else 0.0


class Classification:
    def __init__(self, cfg=None, lab2cname=None, per_class_result=False):
        self._lab2cname = lab2cname
        self._per_class = per_class_result
        self.reset()

    def reset(self):
        self._pred, self._gt = [], []

    def process(self, mo, gt):
        self._pred.append(mo.argmax(1).to(torch.int64))
        self._gt.append(gt.to(torch.int64))

    def preds(self):
        return torch.cat(self._pred).cpu().numpy() if self._pred else np.zeros(0, np.int64)

    def evaluate(self):
        if not self._pred:
            return {"accuracy": 0.0, "error": 100.0, "macro_f1": 0.0}
        return self.evaluate_arrays(torch.cat(self._gt).cpu().numpy(), torch.cat(self._pred).cpu().numpy())

    def evaluate_arrays(self, g, p):
        """evaluator.py:67-125 on host arrays (labels g, predictions p)."""
        g, p = np.asarray(g), np.asarray(p)
        if len(g) == 0:
            return {"accuracy": 0.0, "error": 100.0, "macro_f1": 0.0}
        correct = int((p == g).sum())
        acc = 100.0 * correct / len(g)
        res = {"accuracy": acc, "error": 100.0 - acc, "macro_f1": 100.0 * macro_f1(g, p)}
        print(f"=> result\n* total: {len(g):,}\n* correct: {correct:,}\n* accuracy: {acc:.1f}%\n"
              f"* error: {100 - acc:.1f}%\n* macro_f1: {res['macro_f1']:.1f}%")
        if self._per_class:
            res["per_class"] = {int(c): 100.0 * float(np.mean(p[g == c] == c)) for c in np.unique(g)}
        return res


def base_new_accuracy(preds, labels, n_base):
    """Base / new / harmonic-mean accuracy split (PromptSRC/train.py:335-347)."""
    preds, labels = np.asarray(preds), np.asarray(labels)
    base = labels < n_base
    acc_b = 100.0 * np.mean(preds[base] == labels[base]) if base.any() else 0.0
    acc_n = 100.0 * np.mean(preds[~base] == labels[~base]) if (~base).any() else 0.0
    hm = 2 * acc_b * acc_n / (acc_b + acc_n) if acc_b + acc_n > 0 else 0.0
    return acc_b, acc_n, hm


class LossSummary(dict):
    """The trainers' per-step loss summary (reference: ``{"loss": loss.item()}``,
    PromptSRC/trainers/coop.py:461 / cocoop.py:333) holding detached device scalars and converting them
    on access, so a training step does not stall the host on the GPU every batch; values
    read through ``[]`` / ``items()`` / ``repr`` are the same Python floats."""

    def __setitem__(self, k, v):
        super().__setitem__(k, v.detach() if torch.is_tensor(v) else v)

    def __getitem__(self, k):
        v = super().__getitem__(k)
        return v.item() if torch.is_tensor(v) else v

    def get(self, k, default=None):
        return self[k] if k in self else default

    def items(self):
        return [(k, self[k]) for k in self.keys()]

    def values(self):
        return [self[k] for k in self.keys()]

    def __repr__(self):
        return repr(dict(self.items()))

    __str__ = __repr__
