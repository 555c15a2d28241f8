"""Synthetic DataManager with the Dassl surface the trainers read
(``dm.dataset.classnames``, ``dm.dataset.lab2cname``, ``dm.train_loader_x``,
``dm.test_loader``; batches are dicts {"img", "label"}; data_manager.py:55-162,234-263).

Images are seeded U[0,1) CLIP-normalised tensors, generated once and
kept resident on the device (no decode/augment in the timed region). Labels follow the
imbalanced per-class shot list when given (PER_CLASS_SHOTS), e.g. the repo's
ImageNet-LT setting [16]*500 + [1]*500 (scripts/coop/train.sh:56).
"""
from __future__ import annotations

import numpy as np
import torch

from ..clip import synth


class _Dataset:
    def __init__(self, classnames):
        self.classnames = classnames
        self.lab2cname = {i: c for i, c in enumerate(classnames)}
        self.num_classes = len(classnames)


class SyntheticDataManager:
    def __init__(self, n_cls, resolution, batch_size, n_batches=2, test_batch=100, n_test=0,
                 per_class_shots=None, device="cuda", seed=1, rank=0, n_test_device=0):
        """n_test: test images made on the host (numpy RandomState, as the fixtures);
        n_test_device: a large test set drawn directly in HBM (torch generator on the
        device; U[0,1) then CLIP-normalised), e.g. the 50,000-image eval timing set of
        SURVEY §8(d) -- 30 GB at 224 px fp32, resident, every image distinct."""
        self.dataset = _Dataset(synth.synthetic_classnames(n_cls))
        dev = torch.device(device)
        rs = np.random.RandomState(1000 + seed + 7919 * rank)
        if per_class_shots:
            pool = np.repeat(np.arange(n_cls), per_class_shots)
        else:
            pool = np.arange(n_cls)
        self.train_loader_x = []
        for i in range(n_batches):
            img = synth.make_images(batch_size, resolution, seed=seed + 31 * i + 7919 * rank)
            lab = rs.choice(pool, size=batch_size).astype(np.int64)
            self.train_loader_x.append({"img": torch.from_numpy(img).to(dev),
                                        "label": torch.from_numpy(lab).to(dev)})
        self.test_loader = []
        for i in range(0, n_test, test_batch):
            b = min(test_batch, n_test - i)
            img = synth.make_images(b, resolution, seed=10_000 + seed + i + 7919 * rank)
            lab = rs.randint(0, n_cls, size=b).astype(np.int64)
            self.test_loader.append({"img": torch.from_numpy(img).to(dev),
                                     "label": torch.from_numpy(lab).to(dev)})
        if n_test_device:
            g = torch.Generator(device=dev)
            g.manual_seed(20_000 + seed + 7919 * rank)
            mean = torch.tensor(synth.CLIP_MEAN, device=dev).view(1, 3, 1, 1)
            std = torch.tensor(synth.CLIP_STD, device=dev).view(1, 3, 1, 1)
            for i in range(0, n_test_device, test_batch):
                b = min(test_batch, n_test_device - i)
                img = torch.rand((b, 3, resolution, resolution), generator=g, device=dev).sub_(mean).div_(std)
                lab = torch.randint(0, n_cls, (b,), generator=g, device=dev)
                self.test_loader.append({"img": img, "label": lab})
        self.val_loader = None
