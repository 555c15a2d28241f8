"""MODEL.WEIGHTS_PATH forms (reference clip.py:110-124 / coop.py:165-184):
a torch.save state dict (bare or under "state_dict", loaded weights-only), .npz,
.safetensors and the OpenAI TorchScript archive (read without running its code) all give the
same CLIP state dict, minus the metadata keys build_model drops (model.py:662-705). Files the
loader cannot read safely are refused with an error, never unpickled freely."""
import io
import os
import pickle
import zipfile

import numpy as np
import pytest
import torch

from fsp_amd.clip import synth
from fsp_amd.clip.weights import is_torchscript_archive, load_state_dict


@pytest.fixture(scope="module")
def sd():
    return {k: torch.as_tensor(np.asarray(v)) for k, v in synth.make_state_dict("tiny", seed=0).items()}


def _same(a, b):
    assert set(a) == set(b), set(a) ^ set(b)
    for k in a:
        x, y = torch.as_tensor(np.asarray(a[k])), torch.as_tensor(np.asarray(b[k]))
        assert x.dtype == y.dtype and x.shape == y.shape and torch.equal(x, y), k


def test_torch_save_forms(tmp_path, sd):
    p = tmp_path / "clip.pt"
    torch.save(sd, p)
    _same(load_state_dict(str(p)), sd)
    q = tmp_path / "wrapped.pth.tar"
    torch.save({"state_dict": sd, "epoch": 3}, q)
    _same(load_state_dict(str(q)), sd)
    assert not is_torchscript_archive(str(p))


def test_npz_and_safetensors(tmp_path, sd):
    p = tmp_path / "clip.npz"
    np.savez(p, **{k: v.numpy() for k, v in sd.items()})
    _same(load_state_dict(str(p)), sd)
    from safetensors.torch import save_file
    q = tmp_path / "clip.safetensors"
    save_file({k: v.contiguous() for k, v in sd.items()}, str(q))
    _same(load_state_dict(str(q)), sd)


def test_metadata_keys_dropped(tmp_path, sd):
    p = tmp_path / "meta.pt"
    torch.save(dict(sd, input_resolution=torch.tensor(224), context_length=torch.tensor(77),
                    vocab_size=torch.tensor(49408)), p)
    _same(load_state_dict(str(p)), sd)


class _Node(torch.nn.Module):
    def forward(self, x):
        return x


def _module_tree(sd, dtype):
    """A module whose state_dict() is `sd` (nested by the dotted key path), as the OpenAI
    release's scripted CLIP is, plus its int metadata tensors."""
    root = _Node()
    for key, v in sd.items():
        *path, leaf = key.split(".")
        m = root
        for name in path:
            if not hasattr(m, name):
                m.add_module(name, _Node())
            m = getattr(m, name)
        m.register_parameter(leaf, torch.nn.Parameter(v.to(dtype), requires_grad=False))
    for k, v in (("input_resolution", 224), ("context_length", 77), ("vocab_size", 49408)):
        root.register_buffer(k, torch.tensor(v))
    return root


@pytest.mark.parametrize("dtype", [torch.float32, torch.float16])
def test_torchscript_archive(tmp_path, sd, dtype):
    """torch.jit.save of a traced module tree (the release files' container format: zip with
    <root>/data.pkl, <root>/code/, <root>/data/<storage>): tensors rebuilt from the archive's
    storages, module tree flattened to state_dict() keys, metadata keys dropped."""
    m = _module_tree(sd, dtype)
    ts = torch.jit.trace(m, torch.zeros(1))
    p = tmp_path / "ViT-tiny.pt"
    torch.jit.save(ts, str(p))
    assert is_torchscript_archive(str(p))
    got = load_state_dict(str(p))
    want = {k: v.to(dtype) for k, v in sd.items()}
    _same(got, want)
    # and the same dict torch.jit.load(...).state_dict() gives, minus the metadata
    ref = {k: v for k, v in torch.jit.load(str(p)).state_dict().items()
           if k not in ("input_resolution", "context_length", "vocab_size")}
    _same(got, ref)


def _zip_with_pickle(path, payload):
    with zipfile.ZipFile(path, "w") as zf:
        zf.writestr("m/data.pkl", payload)
        zf.writestr("m/code/__torch__/m.py", "")
        zf.writestr("m/constants.pkl", pickle.dumps(()))


def test_torchscript_archive_refuses_foreign_globals(tmp_path):
    """A data.pkl that names anything but tensor rebuilds, storages and scripted-module
    classes is refused (the global is never resolved, let alone called)."""
    p = tmp_path / "evil.pt"
    _zip_with_pickle(p, b"cos\nsystem\n(S'echo pwned'\ntR.")
    with pytest.raises(pickle.UnpicklingError, match="refusing global os.system"):
        load_state_dict(str(p))


def test_torchscript_archive_without_tensors(tmp_path):
    p = tmp_path / "empty.pt"
    buf = io.BytesIO()
    pickle.dump({"a": 1}, buf, protocol=2)
    _zip_with_pickle(p, buf.getvalue())
    with pytest.raises(ValueError, match="no tensors"):
        load_state_dict(str(p))


class _Foreign:
    pass


def test_plain_pickle_refused(tmp_path):
    """torch.save files go through weights_only=True: arbitrary objects are refused."""
    p = tmp_path / "obj.pt"
    torch.save({"x": _Foreign()}, p)
    with pytest.raises(pickle.UnpicklingError, match="weights_only|Unsupported global"):
        load_state_dict(str(p))


def test_not_a_state_dict(tmp_path):
    p = tmp_path / "list.pt"
    torch.save([torch.zeros(2)], p)
    with pytest.raises(ValueError, match="not a state dict"):
        load_state_dict(str(p))


def test_trainer_uses_weights_path(tmp_path, sd, monkeypatch):
    """load_clip reads MODEL.WEIGHTS_PATH through this loader (CPU check of the plumbing:
    build_model is stubbed, it needs the GPU)."""
    from fsp_amd.engine import trainer as T
    seen = {}
    monkeypatch.setattr(T, "build_model", lambda s, **kw: seen.setdefault("sd", s))
    p = tmp_path / "clip.safetensors"
    from safetensors.torch import save_file
    save_file({k: v.contiguous() for k, v in sd.items()}, str(p))

    class Cfg(dict):
        __getattr__ = dict.__getitem__
    cfg = Cfg(MODEL=Cfg(WEIGHTS_PATH=str(p), BACKBONE=Cfg(NAME="tiny")))
    T.load_clip(cfg, "fp32", torch.device("cpu"))
    _same(seen["sd"], sd)
    os.remove(p)
