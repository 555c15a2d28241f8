"""Helpers shared by the deep-prompt tests: regenerate the seeded initial parameters that
tests/golden/make_golden_deep.py did not store (its _seed_params)."""
import numpy as np
import torch


def seeded_init(meta, shapes):
    """{name: fp32 array} for meta["seeded"] (normal 0.02, RandomState(meta["seed"]), that
    order), meta["half_rounded"] rounded through fp16 as the generator did."""
    rs = np.random.RandomState(meta["seed"])
    out = {}
    for n in meta["seeded"]:
        v = rs.normal(0.0, 0.02, size=tuple(shapes[n])).astype(np.float32)
        if n in meta.get("half_rounded", []):
            v = v.astype(np.float16).astype(np.float32)
        out[n] = v
    return out


def init_params(meta, ref, shapes=None):
    """Every trainable tensor's initial value: stored ones + regenerated seeded ones."""
    vals = {k[len("init_"):]: v for k, v in ref.items() if k.startswith("init_")}
    if meta.get("seeded") and shapes is not None:
        for k, v in seeded_init(meta, shapes).items():
            vals.setdefault(k, v)
    return vals


def grad_of(ref, name):
    """Reference gradient and the row slice it covers (large ones keep their first 32 rows)."""
    if "grad_" + name in ref:
        return ref["grad_" + name], slice(None)
    return ref["grad_" + name + ".rows32"], slice(0, 32)
