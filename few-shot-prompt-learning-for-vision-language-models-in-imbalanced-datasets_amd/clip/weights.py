"""CLIP weight files for ``MODEL.WEIGHTS_PATH`` (the real-weight loader).

The reference gets CLIP through ``clip.load`` / ``load_clip_to_cpu`` (PromptSRC/clip/clip.py:
110-124, trainers/coop.py:165-184): the OpenAI release files are TorchScript archives, read
with ``torch.jit.load`` and turned into a state dict (``model.state_dict()``) for
``build_model`` (clip/model.py:662-705); ``torch.load`` is the fallback for plain state
dicts. Here, without executing anything from the file:

* TorchScript archive (zip with ``<root>/data.pkl`` + ``<root>/code/``): ``data.pkl`` is read
  by a restricted unpickler -- every ``__torch__.*`` class (the scripted modules) becomes an
  attribute record, tensors are rebuilt from the archive's storages, any other global is
  refused -- and the module tree is flattened into the state dict that
  ``model.state_dict()`` returns (``visual.conv1.weight``, ``transformer.resblocks.0...``).
  The TorchScript code in the archive is never compiled or run.
* ``torch.save`` state dicts (optionally under "state_dict"): ``torch.load(weights_only=True)``.
* ``.npz`` (``allow_pickle=False``) and ``.safetensors``.
"""
from __future__ import annotations

import pickle
import zipfile

import numpy as np
import torch

_META_KEYS = ("input_resolution", "context_length", "vocab_size")

_STORAGE_DTYPES = {
    "FloatStorage": torch.float32, "HalfStorage": torch.float16, "BFloat16Storage": torch.bfloat16,
    "DoubleStorage": torch.float64, "LongStorage": torch.int64, "IntStorage": torch.int32,
    "ShortStorage": torch.int16, "CharStorage": torch.int8, "ByteStorage": torch.uint8,
    "BoolStorage": torch.bool,
}


class _Record:
    """A scripted module / object from data.pkl: keeps its attribute state only."""

    qualname = ""
    state = None

    def __init__(self, *args, **kwargs):
        pass

    def __setstate__(self, state):
        self.state = state


class _StorageType:
    def __init__(self, name):
        self.dtype = _STORAGE_DTYPES[name]


def _record_class(qualname):
    return type("Rec", (_Record,), {"qualname": qualname})


class _TorchScriptUnpickler(pickle.Unpickler):
    _ALLOWED = {
        ("torch._utils", "_rebuild_tensor_v2"): torch._utils._rebuild_tensor_v2,
        ("torch._utils", "_rebuild_parameter"): torch._utils._rebuild_parameter,
        ("collections", "OrderedDict"): __import__("collections").OrderedDict,
    }

    def __init__(self, f, zf, root):
        super().__init__(f)
        self.zf, self.root = zf, root
        self._storages = {}

    def find_class(self, module, name):
        if (module, name) in self._ALLOWED:
            return self._ALLOWED[(module, name)]
        if module == "torch" and name in _STORAGE_DTYPES:
            return _StorageType(name)
        if module.startswith("__torch__"):
            return _record_class(module + "." + name)
        raise pickle.UnpicklingError(f"refusing global {module}.{name} in a TorchScript archive")

    def persistent_load(self, pid):
        # ('storage', storage_type, key, location, numel)
        if not (isinstance(pid, tuple) and pid and pid[0] == "storage"):
            raise pickle.UnpicklingError(f"unexpected persistent id {pid!r}")
        st, key = pid[1], str(pid[2])
        dtype = st.dtype if isinstance(st, _StorageType) else torch.float32
        if key not in self._storages:
            raw = self.zf.read(f"{self.root}/data/{key}")
            u8 = torch.frombuffer(bytearray(raw), dtype=torch.uint8) if raw else torch.empty(0, dtype=torch.uint8)
            self._storages[key] = torch.storage.TypedStorage(wrap_storage=u8.untyped_storage(), dtype=dtype,
                                                            _internal=True)
        return self._storages[key]


def _flatten(obj, prefix, out):
    if isinstance(obj, _Record):
        st = obj.state
        if isinstance(st, dict):
            for k, v in st.items():
                if isinstance(k, str) and not k.startswith("_"):
                    _flatten(v, f"{prefix}{k}.", out)
        return
    if isinstance(obj, torch.Tensor):
        out[prefix[:-1]] = obj.detach().clone()


def is_torchscript_archive(path) -> bool:
    if not zipfile.is_zipfile(path):
        return False
    with zipfile.ZipFile(path) as zf:
        names = zf.namelist()
    return any(n.endswith("/constants.pkl") or "/code/" in n for n in names) and \
        any(n.endswith("/data.pkl") for n in names)


def load_torchscript_state_dict(path):
    """State dict of a TorchScript CLIP archive, read without running its code."""
    with zipfile.ZipFile(path) as zf:
        pkl = [n for n in zf.namelist() if n.endswith("/data.pkl") and n.count("/") == 1]
        if not pkl:
            raise ValueError(f"{path}: no <root>/data.pkl in the archive")
        root = pkl[0].split("/")[0]
        import io
        up = _TorchScriptUnpickler(io.BytesIO(zf.read(pkl[0])), zf, root)
        top = up.load()
    sd = {}
    _flatten(top, "", sd)
    if not sd:
        raise ValueError(f"{path}: no tensors found in the TorchScript module tree")
    return sd


def load_state_dict(path):
    """MODEL.WEIGHTS_PATH -> CLIP state dict (tensors / arrays), metadata keys removed."""
    if path.endswith(".npz"):
        with np.load(path, allow_pickle=False) as z:
            sd = {k: z[k] for k in z.files}
    elif path.endswith(".safetensors"):
        from safetensors.torch import load_file
        sd = load_file(path)
    elif is_torchscript_archive(path):
        sd = load_torchscript_state_dict(path)
    else:
        sd = torch.load(path, map_location="cpu", weights_only=True)
        if isinstance(sd, dict) and "state_dict" in sd and isinstance(sd["state_dict"], dict):
            sd = sd["state_dict"]
    if not isinstance(sd, dict):
        raise ValueError(f"{path}: not a state dict")
    return {k: v for k, v in sd.items() if k not in _META_KEYS}
