"""Dassl checkpoint IO (Dassl.pytorch/dassl/utils/torchtools.py:27-157) for the prompt
learners. CoOp / CoCoOp files are readable in both directions with the reference (load and
resume). The deep trainers (IVLP / MaPLe / PromptSRC) register only their prompt parameters,
where the reference registers the whole CustomCLIP: their files load here either way, and
the reference's ``load_model`` (strict=False) reads ours, but the reference's strict resume
of a file written here would report the frozen encoder keys missing.

Layout (save_checkpoint, torchtools.py:27-74): ``<dir>/model.pth.tar-<epoch>`` (or
``model_name``) holding {"state_dict", "epoch", "optimizer", "scheduler", "val_result"},
"module." stripped from the state-dict keys, a ``checkpoint`` pointer file naming the last
file, ``model-best.pth.tar`` copied when ``is_best``.

Loading never executes anything from the file. ``torch.load(weights_only=True)`` reads
plain checkpoints; a reference checkpoint additionally pickles Python objects -- Dassl's
ConstantWarmupScheduler.state_dict() carries its ``successor`` (a CosineAnnealingLR holding
its SGD optimizer, lr_scheduler.py:10-33) -- which the weights-only unpickler refuses. For
those, every global the file names outside the weights-only allowlist is bound to an inert
record class (construction arguments ignored, pickled attribute state kept as data), the file
is read with the same weights-only unpickler, and each record becomes the dict of its
attributes (so a Dassl scheduler's ``successor`` reads as {"last_epoch": ..., ...}).
Tensors, numbers, strings and containers come through unchanged; nothing is called.
"""
from __future__ import annotations

import os
import os.path as osp
import pickle
import shutil
from collections import OrderedDict

import torch


class _Inert:
    """Stand-in for a non-allowlisted global of a checkpoint: ignores construction
    arguments, keeps the pickled attribute state as data, has no behaviour."""

    def __init__(self, *args, **kwargs):
        self._state = None

    def __setstate__(self, state):
        self._state = state

    def __call__(self, *args, **kwargs):
        return _Inert()


def _inert_class(qualname: str):
    return type("Inert_" + qualname.replace(".", "_"), (_Inert,), {"__module__": __name__})


def _plain_dict(*args, **kwargs):
    """collections.defaultdict(...) read as a plain dict (the weights-only unpickler fills
    only dict / OrderedDict / Counter); its default factory is dropped."""
    return {}


# globals that are plain data containers: bound to a dict-returning factory / the builtin
_CONTAINERS = {"collections.defaultdict": _plain_dict, "builtins.dict": dict}


def _scrub(obj):
    """Records -> the dict of their pickled attributes (None when they carried none), stub
    classes -> None, recursively through containers."""
    if isinstance(obj, type) and issubclass(obj, _Inert):
        return None
    if isinstance(obj, _Inert):
        st = getattr(obj, "_state", None)
        if isinstance(st, tuple) and len(st) == 2 and isinstance(st[1], dict):  # (dict, slots)
            st = {**(st[0] or {}), **st[1]}
        return _scrub(st) if isinstance(st, dict) else None
    if isinstance(obj, OrderedDict):
        return OrderedDict((k, _scrub(v)) for k, v in obj.items())
    if isinstance(obj, dict):
        return {k: _scrub(v) for k, v in obj.items()}
    if isinstance(obj, list):
        return [_scrub(v) for v in obj]
    if isinstance(obj, tuple):
        return tuple(_scrub(v) for v in obj)
    return obj


def load_checkpoint(fpath, map_location="cpu"):
    """torchtools.py:77-115 ``load_checkpoint`` without code execution (see module doc)."""
    if fpath is None:
        raise ValueError("File path is None")
    if not osp.exists(fpath):
        raise FileNotFoundError(f'File is not found at "{fpath}"')
    try:
        return torch.load(fpath, map_location=map_location, weights_only=True)
    except pickle.UnpicklingError:
        pass
    names = torch.serialization.get_unsafe_globals_in_checkpoint(fpath)
    stubs = [(_CONTAINERS[n], n) if n in _CONTAINERS else (_inert_class(n), n) for n in names]
    with torch.serialization.safe_globals(stubs):
        ck = torch.load(fpath, map_location=map_location, weights_only=True)
    return _scrub(ck)


def save_checkpoint(state, save_dir, is_best=False, remove_module_from_keys=True, model_name=""):
    """torchtools.py:27-74: writes the file and the ``checkpoint`` pointer; returns the path."""
    os.makedirs(save_dir, exist_ok=True)
    if remove_module_from_keys:
        state["state_dict"] = OrderedDict((k[7:] if k.startswith("module.") else k, v)
                                          for k, v in state["state_dict"].items())
    epoch = state["epoch"]
    if not model_name:
        model_name = "model.pth.tar-" + str(epoch)
    fpath = osp.join(save_dir, model_name)
    torch.save(state, fpath)
    print(f"Checkpoint saved to {fpath}")
    with open(osp.join(save_dir, "checkpoint"), "w+") as f:
        f.write("{}\n".format(osp.basename(fpath)))
    if is_best:
        shutil.copy(fpath, osp.join(osp.dirname(fpath), "model-best.pth.tar"))
    return fpath


def resume_from_checkpoint(fdir, model, optimizer=None, scheduler=None):
    """torchtools.py:118-157: restore weights (+ optimizer, scheduler); returns the epoch.

    The file may hold more than the registered module: the reference's IVLP / MaPLe /
    PromptSRC register a CustomCLIP that also carries the frozen CLIP encoders
    (promptsrc.py:262), where here only the prompt parameters are registered. Keys the module
    does not have are dropped; every key the module has must be in the file (a strict load
    on the module's side, so a CoOp / CoCoOp resume is exactly the reference's)."""
    with open(osp.join(fdir, "checkpoint")) as f:
        fpath = osp.join(fdir, f.readlines()[0].strip("\n"))
    print(f'Loading checkpoint from "{fpath}"')
    ck = load_checkpoint(fpath)
    own = model.state_dict()
    sd = {k: v for k, v in ck["state_dict"].items() if k in own}
    model.load_state_dict(sd)
    if optimizer is not None and ck.get("optimizer") is not None:
        optimizer.load_state_dict(ck["optimizer"])
    if scheduler is not None and ck.get("scheduler") is not None:
        scheduler.load_state_dict(ck["scheduler"])
    return ck["epoch"]
