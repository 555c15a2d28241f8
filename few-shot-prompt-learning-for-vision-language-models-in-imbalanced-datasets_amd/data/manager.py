"""DataManager for the CoOp/CoCoOp trainers over Dassl-style datasets, rank-aware.

Surface of Dassl's DataManager (Dassl.pytorch/dassl/data/data_manager.py:55-162):
``dataset`` (classnames, lab2cname, num_classes), ``train_loader_x``, ``val_loader``,
``test_loader``; batches are dicts {"img", "label", "impath", "index"}
(DatasetWrapper.__getitem__, data_manager.py:234-263). ``dataset`` is any object with the
DatasetBase attributes (train_x, val, test lists of Datum, classnames, lab2cname,
num_classes) -- the readers and few-shot / long-tail splits of data/fewshot.py build one.

The image path: worker processes decode the files (PIL, RGB, as read_image does) into
uint8 arrays; the main process runs the transforms on the GPU (data/preprocess.py, the
CoOp/CoCoOp configs' random_resized_crop / random_flip / normalize for training and
resize / center_crop / normalize for test) and yields device tensors.

Multi-GPU (one process per GPU): the training sampler is built exactly as Dassl builds it
(data/fewshot.py build_sampler: RandomSampler / WeightedClassSampler /
SequentialSampler, torch's global RNG, which dist.sync_rng_from(0) makes identical on every
rank each epoch), so every rank walks the SAME global index stream; it is cut into global
batches of BATCH_SIZE x world (drop_last as the reference: when the set holds a full batch)
and rank r takes its contiguous slice (dist.shard_range). Each batch carries ``n_global``
and ``n_local`` so the trainers weight the gradient all-reduce by the rank's share
(engine/trainer.py). The test split is sharded contiguously; ``TrainerX.test`` gathers the
predictions. CoCoOp class sharding (dist.batches_replicated) instead gives every rank the
whole global batch and the whole test split.

Augmentation: the random-resized-crop / flip parameters come from a generator of the
transform's own (``augment_generator``), not from torch's global RNG -- that one is synced
across ranks every epoch for the sampler stream, so drawing crops from it would give rank r's
k-th image the same crop as rank 0's. Data parallel: one stream per rank (seed + rank);
replicated batches: one stream shared by every rank (they must preprocess identically).
"""
from __future__ import annotations

import numpy as np
import torch
from torch.utils.data import DataLoader, Dataset, Sampler

from .. import dist
from .fewshot import build_sampler


def read_image(path):
    """Dassl read_image (utils/tools.py): PIL open -> RGB, here as uint8 HWC numpy."""
    from PIL import Image
    with Image.open(path) as im:
        return np.asarray(im.convert("RGB"), dtype=np.uint8)


def augment_generator(replicated: bool, seed: int | None = None) -> torch.Generator:
    """CPU generator of the training augmentation stream: seeded from rank 0's torch seed
    (``seed`` overrides it) + this rank's index (data parallel) or + 0 on every rank
    (replicated batches)."""
    base = dist.broadcast_int(torch.initial_seed() if seed is None else seed) & ((1 << 62) - 1)
    g = torch.Generator()
    g.manual_seed(base + (0 if replicated else 1_000_003 * (1 + dist.rank())))
    return g


class ShardedBatchSampler(Sampler):
    """Global batches of batch_size x world from ``sampler``; yields rank r's slice of each
    as a list of (index, global batch size, local batch size) keys. A rank whose slice of a
    short last batch would be empty gets the batch's first item as a pad with local size 0
    (every rank must join the all-reduce; the pad's loss weight is 0)."""

    def __init__(self, sampler, batch_size, drop_last, rank=None, world=None):
        self.sampler = sampler
        self.batch_size = int(batch_size)
        self.drop_last = bool(drop_last)
        self.rank = dist.rank() if rank is None else rank
        self.world = dist.world_size() if world is None else world

    def global_batches(self):
        idx = list(iter(self.sampler))
        G = self.batch_size * self.world
        for b in range(0, len(idx), G):
            chunk = idx[b:b + G]
            if len(chunk) < G and self.drop_last:
                return
            yield chunk

    def __iter__(self):
        for chunk in self.global_batches():
            lo, hi = dist.shard_range(len(chunk), self.rank, self.world)
            if hi > lo:
                yield [(int(i), len(chunk), hi - lo) for i in chunk[lo:hi]]
            else:
                yield [(int(chunk[0]), len(chunk), 0)]

    def __len__(self):
        n = len(self.sampler)
        G = self.batch_size * self.world
        return n // G if self.drop_last else (n + G - 1) // G


class _RangeSampler(Sampler):
    def __init__(self, lo, hi):
        self.lo, self.hi = lo, hi

    def __iter__(self):
        return iter(range(self.lo, self.hi))

    def __len__(self):
        return self.hi - self.lo


class DatasetWrapper(Dataset):
    """data_manager.py:202-275 up to the decoded image (transforms run on the GPU)."""

    def __init__(self, data_source, reader=read_image):
        self.data_source = data_source
        self.reader = reader

    def __len__(self):
        return len(self.data_source)

    def __getitem__(self, key):
        idx, n_global, n_local = key if isinstance(key, tuple) else (key, 0, 0)
        item = self.data_source[idx]
        return {"img": self.reader(item.impath), "label": item.label, "domain": item.domain,
                "impath": item.impath, "index": idx, "n_global": n_global, "n_local": n_local}


def _collate(items):
    return {"img": [it["img"] for it in items],
            "label": torch.tensor([it["label"] for it in items], dtype=torch.int64),
            "domain": torch.tensor([it["domain"] for it in items], dtype=torch.int64),
            "impath": [it["impath"] for it in items],
            "index": torch.tensor([it["index"] for it in items], dtype=torch.int64),
            "n_global": items[0]["n_global"], "n_local": items[0]["n_local"]}


class GpuLoader:
    """Iterates a host DataLoader of decoded images and applies the GPU transform."""

    def __init__(self, loader, transform, device):
        self.loader, self.transform, self.device = loader, transform, device

    def __len__(self):
        return len(self.loader)

    def __iter__(self):
        for b in self.loader:
            out = dict(b)
            out["img"] = self.transform(b["img"])
            out["label"] = b["label"].to(self.device, non_blocking=True)
            yield out


class DataManager:
    def __init__(self, cfg, dataset, device="cuda", reader=read_image, num_workers=None):
        from .preprocess import GpuTransform
        self.dataset = dataset
        self.device = torch.device(device)
        nw = cfg.DATALOADER.NUM_WORKERS if num_workers is None else num_workers
        self.replicated = dist.batches_replicated(cfg)
        rank, world = (0, 1) if self.replicated else (dist.rank(), dist.world_size())

        train = dataset.train_x
        bs = cfg.DATALOADER.TRAIN_X.BATCH_SIZE
        sampler = build_sampler(cfg.DATALOADER.TRAIN_X.SAMPLER, cfg=cfg, data_source=train, batch_size=bs)
        self.train_batch_sampler = ShardedBatchSampler(sampler, bs, drop_last=len(train) >= bs * world,
                                                       rank=rank, world=world)
        self.train_loader_x = GpuLoader(
            DataLoader(DatasetWrapper(train, reader), batch_sampler=self.train_batch_sampler, num_workers=nw,
                       collate_fn=_collate, pin_memory=False),
            GpuTransform(cfg, is_train=True, device=self.device, generator=augment_generator(self.replicated)),
            self.device)

        def test_loader(data):
            if not data:
                return None
            lo, hi = dist.shard_range(len(data), rank, world)
            return GpuLoader(
                DataLoader(DatasetWrapper(data, reader), sampler=_RangeSampler(lo, hi),
                           batch_size=cfg.DATALOADER.TEST.BATCH_SIZE, num_workers=nw, collate_fn=_collate,
                           drop_last=False),
                GpuTransform(cfg, is_train=False, device=self.device), self.device)

        self.val_loader = test_loader(getattr(dataset, "val", None))
        self.test_loader = test_loader(dataset.test)
        self.num_classes = dataset.num_classes
        self.lab2cname = dataset.lab2cname
