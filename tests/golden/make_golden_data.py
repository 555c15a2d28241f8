"""Golden vectors for the few-shot split / class subsampling / sampler semantics, produced by
running the REFERENCE functions themselves on a synthetic item list (this container only):

    python tests/golden/make_golden_data.py

Loaded from their files with minimal stand-ins: ``dassl.data.datasets`` is replaced by a
module holding the real ``dassl.utils.Registry``, a Datum without the file-existence check
and ``DatasetBase = object`` (the real package's __init__ pulls in torchvision/wilds, absent
here); Dassl's ``samplers.py`` and ``base_dataset.py`` (``gdown`` stubbed: used only for
downloads) are loaded by path. Output: tests/golden/data_splits.json (indices only).
"""
from __future__ import annotations

import importlib.util
import json
import os
import random
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference/PromptSRC"
DASSL = "/root/reference/Dassl.pytorch"


def _load(name, path):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


class Item:
    def __init__(self, impath="", label=0, domain=0, classname=""):
        self.impath, self.label, self.domain, self.classname = impath, label, domain, classname


def items(labels, tag):
    return [Item(f"{tag}{i}", int(y), 0, f"class{int(y)}") for i, y in enumerate(labels)]


def ids(seq):
    return [int(it.impath[1:]) for it in seq]


def main():
    sys.path.insert(0, DASSL)
    sys.path.insert(0, REF)
    from dassl.utils import Registry
    fake_data = types.ModuleType("dassl.data")
    fake_ds = types.ModuleType("dassl.data.datasets")
    fake_ds.DATASET_REGISTRY = Registry("DATASET")
    fake_ds.Datum = Item
    fake_ds.DatasetBase = object
    sys.modules["dassl.data"] = fake_data
    sys.modules["dassl.data.datasets"] = fake_ds
    sys.modules["gdown"] = types.ModuleType("gdown")
    from datasets import imagenet, oxford_pets  # PromptSRC/datasets (empty package __init__)
    samplers = _load("ref_samplers", os.path.join(DASSL, "dassl/data/samplers.py"))
    base = _load("ref_base_dataset", os.path.join(DASSL, "dassl/data/datasets/base_dataset.py"))

    rs = np.random.RandomState(0)
    n_cls = 40
    counts = rs.randint(1, 31, size=n_cls)
    train_labels = rs.permutation(np.repeat(np.arange(n_cls), counts))
    test_labels = rs.permutation(np.repeat(np.arange(n_cls), rs.randint(2, 9, size=n_cls)))
    train, test = items(train_labels, "t"), items(test_labels, "v")
    per_class = [16] * 20 + [1] * 20
    out = {"train_labels": train_labels.tolist(), "test_labels": test_labels.tolist(), "per_class": per_class}

    IN = imagenet.ImageNet
    random.seed(1)
    out["imagenet_uniform16"] = {"train": ids(IN.generate_fewshot_dataset(train, num_shots=16)),
                                 "test": ids(IN.generate_fewshot_dataset(test, num_shots=4))}
    random.seed(1)
    out["imagenet_per_class"] = {"train": ids(IN.generate_per_class_fewshot_dataset(train, per_class)),
                                 "test": ids(IN.generate_per_class_fewshot_dataset(test, [min(s, 4) for s in per_class]))}
    random.seed(2)
    out["imagenet_per_class_short"] = ids(IN.generate_per_class_fewshot_dataset(train, per_class[:30]))
    OP = oxford_pets.OxfordPets
    random.seed(5)
    out["pets_per_class"] = ids(OP.generate_per_class_fewshot_dataset(train, per_class))
    random.seed(5)
    out["pets_uniform2"] = ids(OP.generate_fewshot_dataset(train, num_shots=2))
    db = base.DatasetBase.__new__(base.DatasetBase)
    random.seed(3)
    out["dassl_fewshot4"] = ids(db.generate_fewshot_dataset(train, num_shots=4))
    random.seed(3)
    out["dassl_fewshot8_repeat"] = ids(db.generate_fewshot_dataset(train, num_shots=8, repeat=True))
    random.seed(3)
    a, b = db.generate_fewshot_dataset(train, test, num_shots=2)
    out["dassl_fewshot2_two_sources"] = [ids(a), ids(b)]
    for sub in ("base", "new"):
        tr, te = OP.subsample_classes(train, test, subsample=sub)
        out[f"subsample_{sub}"] = {"train": [[int(x.impath[1:]), x.label] for x in tr],
                                   "test": [[int(x.impath[1:]), x.label] for x in te]}
    torch.manual_seed(0)
    s = samplers.WeightedClassSampler(train, replacement=True, num_samples=64)
    out["weighted_sampler_seed0"] = {"weights": s.weights, "indices": [int(i) for i in s]}
    with open(os.path.join(HERE, "data_splits.json"), "w") as f:
        json.dump(out, f)
    print("wrote data_splits.json")


if __name__ == "__main__":
    main()
