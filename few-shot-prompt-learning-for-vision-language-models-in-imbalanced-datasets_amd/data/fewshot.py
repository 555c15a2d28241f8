"""Few-shot / long-tail ("imbalanced") split construction, base/new class subsampling and
the class-balanced sampler, with the reference's RNG semantics (same seed -> same images).

* ``generate_fewshot_dataset`` -- uniform K-shot: per label in first-appearance order,
  ``random.shuffle`` the label's indices and keep the first K
  (PromptSRC/datasets/imagenet.py:149-162, oxford_pets.py:256-269).
* ``generate_per_class_fewshot_dataset`` -- the imbalanced setting: label y keeps
  ``shots_per_class[y]`` items (imagenet.py:164-186; labels past the list keep 0 there,
  while oxford_pets.py:239-253 raises IndexError -- ``strict=True``).
* ``dassl_generate_fewshot_dataset`` -- Dassl's ``DatasetBase.generate_fewshot_dataset``
  (``random.sample`` / ``random.choices`` with repeat; base_dataset.py:167-209).
* ``build_fewshot_splits`` -- the ImageNet flow (imagenet.py:44-116): ``random.seed(seed)``
  once, then train, then test at ``min(shots, 4)`` per class.
* ``subsample_classes`` -- base / new halves with relabelling (oxford_pets.py:198-237).
* ``WeightedClassSampler`` -- weight 1 / count(label) per item through torch's
  ``WeightedRandomSampler`` (Dassl samplers.py:181-212): same torch RNG stream, same indices.
"""
from __future__ import annotations

import math
import random
from collections import Counter, defaultdict

from torch.utils.data.sampler import RandomSampler, Sampler, SequentialSampler, WeightedRandomSampler


class Datum:
    """Dassl Datum (base_dataset.py:11-50) without the file-existence assertion (synthetic
    items carry no file)."""

    def __init__(self, impath="", label=0, domain=0, classname=""):
        if not isinstance(impath, str):
            raise AssertionError("impath must be a str")
        self._impath, self._label, self._domain, self._classname = impath, label, domain, classname

    impath = property(lambda self: self._impath)
    label = property(lambda self: self._label)
    domain = property(lambda self: self._domain)
    classname = property(lambda self: self._classname)

    def __repr__(self):
        return f"Datum({self._impath!r}, {self._label}, {self._classname!r})"


def _tracker(dataset):
    t = defaultdict(list)
    for idx, item in enumerate(dataset):
        t[item.label].append(idx)
    return t


def generate_fewshot_dataset(dataset, num_shots=1):
    out = []
    for _, idxs in _tracker(dataset).items():
        random.shuffle(idxs)
        out.extend(dataset[i] for i in idxs[:num_shots])
    return out


def generate_per_class_fewshot_dataset(dataset, shots_per_class, strict=False):
    out = []
    for label, idxs in _tracker(dataset).items():
        if strict:
            n = shots_per_class[label]
        else:
            n = shots_per_class[label] if label < len(shots_per_class) else 0
        random.shuffle(idxs)
        out.extend(dataset[i] for i in idxs[:n])
    return out


def dassl_generate_fewshot_dataset(*data_sources, num_shots=-1, repeat=False):
    if num_shots < 1:
        return data_sources[0] if len(data_sources) == 1 else data_sources
    output = []
    for src in data_sources:
        groups = defaultdict(list)
        for item in src:
            groups[item.label].append(item)
        ds = []
        for _, items in groups.items():
            if len(items) >= num_shots:
                ds.extend(random.sample(items, num_shots))
            elif repeat:
                ds.extend(random.choices(items, k=num_shots))
            else:
                ds.extend(items)
        output.append(ds)
    return output[0] if len(output) == 1 else output


def build_fewshot_splits(train, test, num_shots, per_class_shots, seed):
    """(train, test) after the ImageNet few-shot logic of imagenet.py:44-108."""
    random.seed(seed)
    if num_shots > 0:
        train = generate_fewshot_dataset(train, num_shots=num_shots)
        test = generate_fewshot_dataset(test, num_shots=min(num_shots, 4))
    elif num_shots < 0 and len(per_class_shots) > 0:
        test_shots = [min(s, 4) for s in per_class_shots]
        train = generate_per_class_fewshot_dataset(train, per_class_shots)
        test = generate_per_class_fewshot_dataset(test, test_shots)
    return train, test


def subsample_classes(*args, subsample="all"):
    if subsample not in ("all", "base", "new"):
        raise AssertionError(subsample)
    if subsample == "all":
        return args
    labels = sorted({item.label for item in args[0]})
    m = math.ceil(len(labels) / 2)
    selected = labels[:m] if subsample == "base" else labels[m:]
    relabel = {y: i for i, y in enumerate(selected)}
    return [[Datum(impath=it.impath, label=relabel[it.label], classname=it.classname)
             for it in ds if it.label in relabel] for ds in args]


class WeightedClassSampler(Sampler):
    """Every class equally likely: item weight 1 / count(item.label)."""

    def __init__(self, data_source, replacement=True, num_samples=None):
        self.data_source = data_source
        self.replacement = replacement
        self.num_samples = len(data_source) if num_samples is None else num_samples
        count = Counter(item.label for item in data_source)
        self.weights = [1.0 / count[item.label] for item in data_source]
        self.w_sampler = WeightedRandomSampler(weights=self.weights, num_samples=self.num_samples,
                                               replacement=self.replacement)

    def __iter__(self):
        return iter(self.w_sampler)

    def __len__(self):
        return self.num_samples


def build_sampler(sampler_type, cfg=None, data_source=None, batch_size=32, replacement=True,
                  num_samples=None):
    """samplers.py:215-249 for the samplers the CoOp/CoCoOp scripts use."""
    if sampler_type == "RandomSampler":
        return RandomSampler(data_source)
    if sampler_type == "SequentialSampler":
        return SequentialSampler(data_source)
    if sampler_type == "WeightedClassSampler":
        return WeightedClassSampler(data_source, replacement=replacement, num_samples=num_samples)
    raise ValueError(f"Unknown sampler type: {sampler_type}")
