"""Few-shot / long-tail split construction, base/new subsampling and the class-balanced
sampler vs golden vectors produced by the REFERENCE functions (tests/golden/
make_golden_data.py: imagenet.py, oxford_pets.py, Dassl base_dataset.py / samplers.py on a
synthetic 40-class item list). Exact index equality (integer work)."""
import json
import os
import random

import torch

from fsp_amd.data import fewshot as F

GOLD = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "data_splits.json")))


def _items(labels, tag):
    return [F.Datum(f"{tag}{i}", int(y), 0, f"class{int(y)}") for i, y in enumerate(labels)]


TRAIN = _items(GOLD["train_labels"], "t")
TEST = _items(GOLD["test_labels"], "v")
PER_CLASS = GOLD["per_class"]


def ids(seq):
    return [int(it.impath[1:]) for it in seq]


def test_imagenet_uniform_and_per_class_flows():
    tr, te = F.build_fewshot_splits(TRAIN, TEST, 16, [], seed=1)
    assert ids(tr) == GOLD["imagenet_uniform16"]["train"]
    assert ids(te) == GOLD["imagenet_uniform16"]["test"]
    tr, te = F.build_fewshot_splits(TRAIN, TEST, -1, PER_CLASS, seed=1)
    assert ids(tr) == GOLD["imagenet_per_class"]["train"]
    assert ids(te) == GOLD["imagenet_per_class"]["test"]
    # the long tail really is imbalanced: head classes 16 (or all), tail classes 1
    counts = torch.bincount(torch.tensor([it.label for it in tr]), minlength=40)
    assert all(int(c) <= s for c, s in zip(counts, PER_CLASS)) and int(counts[20:].max()) == 1


def test_per_class_short_list_and_strict():
    random.seed(2)
    assert ids(F.generate_per_class_fewshot_dataset(TRAIN, PER_CLASS[:30])) == GOLD["imagenet_per_class_short"]
    random.seed(5)
    assert ids(F.generate_per_class_fewshot_dataset(TRAIN, PER_CLASS, strict=True)) == GOLD["pets_per_class"]
    random.seed(5)
    assert ids(F.generate_fewshot_dataset(TRAIN, num_shots=2)) == GOLD["pets_uniform2"]
    try:
        F.generate_per_class_fewshot_dataset(TRAIN, PER_CLASS[:30], strict=True)
    except IndexError:
        pass
    else:
        raise AssertionError("oxford_pets semantics raise IndexError on a short shot list")


def test_dassl_generate_fewshot_dataset():
    random.seed(3)
    assert ids(F.dassl_generate_fewshot_dataset(TRAIN, num_shots=4)) == GOLD["dassl_fewshot4"]
    random.seed(3)
    assert ids(F.dassl_generate_fewshot_dataset(TRAIN, num_shots=8, repeat=True)) == GOLD["dassl_fewshot8_repeat"]
    random.seed(3)
    a, b = F.dassl_generate_fewshot_dataset(TRAIN, TEST, num_shots=2)
    assert [ids(a), ids(b)] == GOLD["dassl_fewshot2_two_sources"]
    assert F.dassl_generate_fewshot_dataset(TRAIN, num_shots=0) is TRAIN


def test_subsample_base_new():
    for sub in ("base", "new"):
        tr, te = F.subsample_classes(TRAIN, TEST, subsample=sub)
        assert [[int(x.impath[1:]), x.label] for x in tr] == GOLD[f"subsample_{sub}"]["train"]
        assert [[int(x.impath[1:]), x.label] for x in te] == GOLD[f"subsample_{sub}"]["test"]
    assert F.subsample_classes(TRAIN, TEST, subsample="all") == (TRAIN, TEST)


def test_weighted_class_sampler():
    torch.manual_seed(0)
    s = F.build_sampler("WeightedClassSampler", data_source=TRAIN, num_samples=64)
    assert s.weights == GOLD["weighted_sampler_seed0"]["weights"]
    assert [int(i) for i in s] == GOLD["weighted_sampler_seed0"]["indices"]
    assert len(s) == 64
