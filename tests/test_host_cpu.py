"""CPU: host-side logic (no GPU compute): the C-ABI library loads and exports every
symbol include/clipk.h declares, prompt slot tables reproduce the reference prompt
layouts, tokenizer, config, registry, losses' alpha, metrics, the fp32s LN-fold table contract."""
import json
import os
import re

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    src = open(os.path.join(ROOT, "include", "clipk.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(clipk_\w+)\s*\(", src)))


def test_library_exports_every_header_symbol():
    from fsp_amd import _native
    lib = _native.load()
    names = header_functions()
    assert len(names) >= 30
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    assert set(names) == set(_native.SIGNATURES), set(names) ^ set(_native.SIGNATURES)
    assert lib.clipk_version().decode().startswith("clipk")
    assert "shape" in _native.strerror(-2)


def test_library_is_built_from_this_tree():
    """libclipk.so embeds the digest of the sources it was built from (clipk_source_digest); the
    loader compares it with the tree it ships with."""
    from fsp_amd import _native
    _native.load()
    assert _native.library_digest() == _native.source_digest()
    rels = [r for r, _ in _native.source_files()]
    assert "csrc/gemm.hip" in rels and "csrc/Makefile" in rels and rels[-1] == "include/clipk.h"


def test_stale_library_is_refused(monkeypatch, tmp_path):
    """A library whose embedded digest differs from the tree (a stale build) does not load."""
    from fsp_amd import _native
    monkeypatch.setattr(_native, "_lib", None)
    monkeypatch.setattr(_native, "source_digest", lambda: "0" * 64)
    with pytest.raises(_native.ClipkError, match="built from other sources"):
        _native.load()
    # and the digest really follows the sources: one byte changed in a copy changes it
    src = tmp_path / "gemm.hip"
    orig = dict(_native.source_files())["csrc/gemm.hip"]
    src.write_bytes(open(orig, "rb").read() + b"\n")
    monkeypatch.undo()
    built = _native.library_digest()  # loads the real library first (the tree's digest)
    files = [(r, str(src) if r == "csrc/gemm.hip" else p) for r, p in _native.source_files()]
    monkeypatch.setattr(_native, "source_files", lambda: files)
    assert _native.source_digest() != built


def test_gemm_config_knob_range():
    """The GEMM tile knob accepts the shipped configurations only (7 = the round-3 64x128
    small-M tile); the variants measured slower (4 / 5: 64-B rows, 8 / 9: deep-A ring; round 2's
    8-phase ping-pong, once cfg 7) left the build."""
    from fsp_amd import _native
    lib = _native.load()
    try:
        for cfg in (-1, 0, 1, 2, 3, 6, 7):
            assert lib.clipk_gemm_set_config(cfg) == 0, cfg
        for cfg in (-2, 4, 5, 8, 9, 10):
            assert lib.clipk_gemm_set_config(cfg) == -1, cfg
    finally:
        lib.clipk_gemm_set_config(-1)


def test_missing_library_fails_loudly(monkeypatch):
    from fsp_amd import _native
    monkeypatch.setattr(_native, "_lib", None)
    monkeypatch.setattr(_native, "LIB_PATH", "/nonexistent/libclipk.so")
    with pytest.raises(_native.ClipkError):
        _native.load()


def test_ops_refuse_cpu_tensors():
    from fsp_amd import ops, _native
    with pytest.raises(_native.ClipkError):
        ops.gemm(torch.zeros(4, 64, dtype=torch.float16), torch.zeros(128, 64, dtype=torch.float16))


@pytest.mark.parametrize("position", ["end", "middle", "front"])
@pytest.mark.parametrize("csc", [False, True])
def test_prompt_layout_matches_reference_cat(position, csc):
    from oracle import clip_oracle as O
    from fsp_amd.trainers._fns import prompt_layout
    rs = np.random.RandomState(0)
    C, n_ctx, W = 6, 4, 8
    name_lens = [1, 2, 3, 1, 4, 2]
    eot = [1 + n_ctx + nl + 1 for nl in name_lens]
    emb = torch.from_numpy(rs.randn(C, 77, W).astype(np.float32))
    ctx = torch.from_numpy(rs.randn(*((C, n_ctx, W) if csc else (n_ctx, W))).astype(np.float32))
    ref = O.coop_prompts(ctx, emb[:, :1], emb[:, 1 + n_ctx:], name_lens, position).numpy()
    src, cpos, L = prompt_layout(C, n_ctx, name_lens, position, eot, truncate=True)
    assert L == max(eot) + 1
    out = np.zeros((C, L, W), np.float32)
    for c in range(C):
        for t in range(L):
            m = src[c, t]
            cv = ctx[c] if csc else ctx
            out[c, t] = emb[c, m].numpy() if m >= 0 else cv[-1 - m].numpy()
            if m < 0:
                assert cpos[c, -1 - m] == t
    np.testing.assert_array_equal(out, ref[:, :L])
    # the EOT token sits at the tokenized argmax position in every layout
    for c in range(C):
        assert src[c, eot[c]] == eot[c]


REF_VOCAB = "/root/reference/PromptSRC/clip/bpe_simple_vocab_16e6.txt.gz"  # build container only


def test_tokenizer_matches_reference_probes():
    """The BPE merge loop vs token ids the reference's SimpleTokenizer produced (fixture),
    with the vocab file passed explicitly: the product never searches the reference checkout
    (find_vocab looks at $FSP_BPE_VOCAB and the package directory only)."""
    from fsp_amd.clip.tokenizer import BPETokenizer, find_vocab
    probes = json.load(open(os.path.join(ROOT, "tests", "golden", "tokenizer_probes.json")))
    path = find_vocab() or (REF_VOCAB if os.path.isfile(REF_VOCAB) else None)
    if path is None:
        pytest.skip("BPE vocab not available (no $FSP_BPE_VOCAB, reference checkout absent)")
    tok = BPETokenizer(path)
    for s, ids in probes.items():
        assert tok.encode(s) == ids, s


def test_tokenizer_fallback_table_covers_synthetic_prompts():
    from fsp_amd.clip.tokenizer import BPETokenizer
    tok = BPETokenizer.__new__(BPETokenizer)
    tok.encoder = None
    tok._fallback = json.load(open(os.path.join(
        ROOT, "few-shot-prompt-learning-for-vision-language-models-in-imbalanced-datasets_amd", "clip",
        "bpe_fallback.json")))
    probes = json.load(open(os.path.join(ROOT, "tests", "golden", "tokenizer_probes.json")))
    for s in ["X X X X class7.", "a photo of a class123.", "X " * 16 + "class999."]:
        assert tok.encode(s) == probes[s]
    with pytest.raises(KeyError, match="FSP_BPE_VOCAB"):
        tok.encode("a photo of a dog.")


def test_tokenizer_never_searches_the_reference(monkeypatch):
    from fsp_amd.clip import tokenizer as T
    monkeypatch.delenv("FSP_BPE_VOCAB", raising=False)
    assert all("/root/reference" not in c for c in T._vocab_candidates())


def test_tokenize_matches_golden_tokens():
    from fsp_amd.clip.tokenizer import tokenize
    from parity_util import load_fixture
    meta, ref = load_fixture("cocoop_vitb16_c4")
    names = [f"class{i}" for i in range(meta["n_cls"])]
    toks = tokenize([meta["ctx_init"] + " " + n + "." for n in names])
    np.testing.assert_array_equal(toks, ref["tokenized"])
    with pytest.raises(RuntimeError):
        tokenize("x " * 100)
    assert tokenize("x " * 100, truncate=True)[0, -1] == 49407


def test_config_merge_and_freeze(tmp_path):
    from fsp_amd.engine.config import get_cfg_default
    cfg = get_cfg_default()
    y = tmp_path / "c.yaml"
    y.write_text("TRAINER:\n  COCOOP:\n    N_CTX: 4\n    CTX_INIT: 'a photo of a'\nOPTIM:\n  LR: 0.002\n"
                 "INPUT:\n  SIZE: (224, 224)\n")
    cfg.merge_from_file(str(y))
    cfg.merge_from_list(["TRAINER.COOP.CSC", "True", "DATASET.PER_CLASS_SHOTS", "[16, 1]", "OPTIM.MAX_EPOCH", "5"])
    assert cfg.TRAINER.COCOOP.N_CTX == 4 and cfg.TRAINER.COOP.CSC is True
    assert cfg.DATASET.PER_CLASS_SHOTS == [16, 1] and cfg.OPTIM.MAX_EPOCH == 5
    assert cfg.TRAINER.COOP.get("LOSS_TYPE", "ce") == "ce"
    cfg.freeze()
    with pytest.raises(AttributeError):
        cfg.SEED = 3


def test_registry_semantics():
    from fsp_amd.engine.registry import Registry, TRAINER_REGISTRY
    import fsp_amd.trainers  # noqa: F401
    assert {"CoOp", "CoCoOp"} <= set(TRAINER_REGISTRY.registered_names())
    r = Registry("X")

    @r.register()
    class A:
        pass
    with pytest.raises(KeyError):
        r.register(A)
    with pytest.raises(KeyError):
        r.get("B")


def test_focal_alpha_semantics():
    from fsp_amd.trainers.losses import focal_alpha
    assert focal_alpha([4, 1, 2, 0, 3], 5, zero_guard=True)[3] == 0.0
    with pytest.raises(ZeroDivisionError):
        focal_alpha([4, 0], 2, zero_guard=False)
    assert focal_alpha("[2,2]", 2, True) == [1.0, 1.0]
    assert focal_alpha([], 2, True) is None


def test_metrics_match_sklearn():
    from sklearn.metrics import f1_score
    from fsp_amd.engine.metrics import macro_f1, compute_accuracy, base_new_accuracy
    rs = np.random.RandomState(0)
    y, p = rs.randint(0, 7, 200), rs.randint(0, 7, 200)
    assert abs(macro_f1(y, p) - f1_score(y, p, average="macro", labels=np.unique(y))) < 1e-12
    # Dassl's evaluator averages over the labels present in y_true only (evaluator.py:71-76):
    # a class that is only ever predicted must not add an F1 of 0
    y2, p2 = rs.randint(0, 5, 100), rs.randint(0, 7, 100)
    assert set(p2) - set(y2)
    ref = f1_score(y2, p2, average="macro", labels=np.unique(y2))
    assert abs(macro_f1(y2, p2) - ref) < 1e-12
    assert macro_f1(y2, p2) != f1_score(y2, p2, average="macro")
    logits = torch.from_numpy(rs.randn(10, 5))
    lab = torch.from_numpy(rs.randint(0, 5, 10))
    acc = compute_accuracy(logits, lab)[0].item()
    assert abs(acc - 100 * (logits.argmax(1) == lab).double().mean().item()) < 1e-4
    b, n, hm = base_new_accuracy(np.array([0, 1, 3, 3]), np.array([0, 2, 3, 2]), 2)
    assert b == 100.0 and abs(n - 100 / 3) < 1e-9 and abs(hm - 2 * 100 * (100 / 3) / (100 + 100 / 3)) < 1e-9


@pytest.mark.parametrize("position,n_ctx,P_expect", [("end", 4, 5), ("end", 16, 16), ("middle", 8, 5),
                                                     ("front", 4, None)])
def test_shared_prefix_tables_reconstruct_prompts(position, n_ctx, P_expect):
    """Packed rows (prefix once per group + each class's rows P..EOT) hold exactly the
    reference prompt tokens; ctx slot row lists cover every packed row using the slot."""
    from oracle import clip_oracle as O
    from fsp_amd.trainers._fns import prompt_layout
    from fsp_amd.trainers.prompt_base import shared_prefix_tables
    rs = np.random.RandomState(1)
    C, W = 7, 8
    name_lens = [1, 2, 3, 1, 4, 2, 5]
    eot = [1 + n_ctx + nl + 1 for nl in name_lens]
    emb = torch.from_numpy(rs.randn(C, 77, W).astype(np.float32))
    emb[:, 0] = emb[0, 0]  # SOT token embedding is class independent
    ctx = torch.from_numpy(rs.randn(n_ctx, W).astype(np.float32))
    ref = O.coop_prompts(ctx, emb[:, :1], emb[:, 1 + n_ctx:], name_lens, position).numpy()
    src, cpos, L = prompt_layout(C, n_ctx, name_lens, position, eot, truncate=True)
    pk = shared_prefix_tables(src, cpos, eot, n_ctx, csc=False)
    if P_expect is None:
        assert pk is None
        return
    P, R, seg, row_tab = pk["P"], pk["R"], pk["seg"], pk["row_tab"]
    assert P == P_expect and R == P + sum(e + 1 - P for e in eot)
    packed = np.zeros((R, W), np.float32)  # numpy restatement of clipk_prompt_assemble_rows
    for r in range(R):
        c, t = divmod(int(row_tab[r]), L)
        m = src[c, t]
        packed[r] = emb[c, m].numpy() if m >= 0 else ctx[-1 - m].numpy()
    for c in range(C):
        off, qn = seg[c]
        assert off + qn - 1 == pk["eot_in_group"][c] and qn == eot[c] + 1 - P
        seq = np.concatenate([packed[:P], packed[off:off + qn]])
        np.testing.assert_array_equal(seq, ref[c, :eot[c] + 1])
    for k in range(n_ctx):
        rows = sorted(pk["slot_rows"][pk["slot_ptr"][k]:pk["slot_ptr"][k + 1]].tolist())
        expect = sorted(r for r in range(R) if src.flat[row_tab[r]] == -1 - k)
        assert rows == expect
    # attention tiles: cover the class rows in order, <= 16 rows, whole classes only
    tiles, rf = pk["tiles"], pk["row_first"]
    starts = {int(o) for o, _ in seg}
    assert tiles[0][0] == P and sum(int(n) for _, n in tiles) == R - P
    for (t0, n), nxt in zip(tiles, list(tiles[1:]) + [(R, 0)]):
        assert 1 <= n <= 16 and t0 + n == nxt[0] and t0 in starts and (t0 + n == R or t0 + n in starts)
    for c in range(C):
        off, qn = seg[c]
        assert (rf[off:off + qn] == off).all()
    assert (rf[:P] == 0).all()
    # CSC contexts and over-long class suffixes fall back to the plain layout
    assert shared_prefix_tables(src, cpos, eot, n_ctx, csc=True) is None
    assert shared_prefix_tables(src, cpos, [e + 20 for e in eot], n_ctx, csc=False) is None


class _CpuLogits(torch.nn.Module):
    """Test double for a CustomCLIP on CPU: logits = image.flatten(1) @ proj."""

    def __init__(self, proj):
        super().__init__()
        self.proj = proj

    def forward(self, x):
        return x.reshape(x.shape[0], -1) @ self.proj


def _dummy_trainer(tmp_path, test_batches=None, n_ctx=4, W=8, C=3):
    import torch.nn as nn
    from fsp_amd.engine.config import get_cfg_default
    from fsp_amd.engine.optim import build_optimizer, build_lr_scheduler
    from fsp_amd.engine.trainer import TrainerX

    class Learner(nn.Module):
        def __init__(self):
            super().__init__()
            self.ctx = nn.Parameter(torch.zeros(n_ctx, W))
            self.register_buffer("token_prefix", torch.ones(C, 1, W))
            self.register_buffer("token_suffix", torch.ones(C, 72, W))

    class Dummy(TrainerX):
        def build_model(self):
            self.learner = Learner()
            self.model = _CpuLogits(torch.from_numpy(np.random.RandomState(0).randn(12, C).astype(np.float32)))
            self.optim = build_optimizer(self.learner, self.cfg.OPTIM)
            self.sched = build_lr_scheduler(self.optim, self.cfg.OPTIM)
            self.register_model("prompt_learner", self.learner, self.optim, self.sched)

    cfg = get_cfg_default()
    cfg.OUTPUT_DIR = str(tmp_path)
    cfg.OPTIM.MAX_EPOCH = 2
    cfg.OPTIM.WARMUP_EPOCH = 1
    cfg.OPTIM.WARMUP_TYPE = "constant"

    class DM:
        test_loader = test_batches or []
        val_loader = None
    return Dummy(cfg, dm=DM())


def test_trainer_test_contract(tmp_path):
    """TrainerX.test follows Dassl (trainer.py:446-486): (y_true, y_pred) numpy arrays with
    return_pred (PromptSRC/train.py:328,356 unpack it), otherwise the first metric (accuracy)
    as a float; the split defaults to cfg.TEST.SPLIT."""
    from sklearn.metrics import f1_score
    rs = np.random.RandomState(3)
    batches = [{"img": torch.from_numpy(rs.randn(5, 3, 2, 2).astype(np.float32)),
                "label": torch.from_numpy(rs.randint(0, 3, 5))} for _ in range(3)]
    t = _dummy_trainer(tmp_path, batches)
    y_true, y_pred = t.test(return_pred=True)
    assert isinstance(y_true, np.ndarray) and isinstance(y_pred, np.ndarray)
    ref_pred = np.concatenate([t.model(b["img"]).argmax(1).numpy() for b in batches])
    np.testing.assert_array_equal(y_true, np.concatenate([b["label"].numpy() for b in batches]))
    np.testing.assert_array_equal(y_pred, ref_pred)
    acc = t.test()
    assert isinstance(acc, float) and abs(acc - 100.0 * np.mean(y_true == y_pred)) < 1e-9
    res = t.evaluator.evaluate_arrays(y_true, y_pred)
    assert list(res)[:3] == ["accuracy", "error", "macro_f1"]
    assert abs(res["macro_f1"] - 100 * f1_score(y_true, y_pred, average="macro", labels=np.unique(y_true))) < 1e-9
    assert t.cfg.TEST.SPLIT == "test"


def test_reference_checkpoint_resume(tmp_path):
    """A checkpoint written by the REFERENCE's own save_model / save_checkpoint
    (tests/golden/make_golden_trainer.py: Dassl TrainerBase.save_model after 2 epochs of
    CoOp, scheduler = ConstantWarmupScheduler whose state pickles its CosineAnnealingLR
    successor) resumes here: weights, SGD momentum state and the epoch / LR position."""
    import shutil
    from parity_util import load_fixture
    meta, ref = load_fixture("trainer_coop")
    src = os.path.join(ROOT, "tests", "golden", "ref_ckpt_coop")
    shutil.copytree(src, tmp_path / "out")
    t = _dummy_trainer(tmp_path, n_ctx=4, W=128, C=5)
    start = t.resume_model_if_exist(str(tmp_path / "out"))
    assert start == meta["epochs"] == 2
    np.testing.assert_array_equal(t.learner.ctx.detach().numpy(), ref["ctx_final"])
    assert abs(t.get_current_lr() - ref["lr_after_epoch"][-1]) < 1e-15
    st = t.optim.state[t.learner.ctx]
    assert st["momentum_buffer"].shape == (4, 128)
    g = t.optim.param_groups[0]
    assert g["momentum"] == 0.9 and g["weight_decay"] == 5e-4 and g["dampening"] == 0


def test_checkpoint_shapes_match_reference(tmp_path):
    """Our checkpoints have the reference's shape: the optimizer state loads into
    torch.optim.SGD (same param-group keys), the scheduler state has the keys of Dassl's
    ConstantWarmupScheduler (a CosineAnnealingLR successor advanced past warmup; the
    wrapper's count saturates at WARMUP_EPOCH), and the file reads back here."""
    from fsp_amd.engine import checkpoint as C
    ref = C.load_checkpoint(os.path.join(ROOT, "tests", "golden", "ref_ckpt_coop", "prompt_learner",
                                         "model.pth.tar-2"))
    t = _dummy_trainer(tmp_path, n_ctx=4, W=128, C=5)
    t.learner.ctx.grad = torch.ones_like(t.learner.ctx)
    t.update_lr()
    t.update_lr()
    t.save_model(1, str(tmp_path / "ours"))
    ours = C.load_checkpoint(str(tmp_path / "ours" / "prompt_learner" / "model.pth.tar-2"))
    assert set(ours) == set(ref)
    assert set(ours["state_dict"]) == set(ref["state_dict"])
    assert set(ours["optimizer"]["param_groups"][0]) == set(ref["optimizer"]["param_groups"][0])
    assert set(ours["scheduler"]) == set(ref["scheduler"])
    assert ours["scheduler"]["last_epoch"] == ref["scheduler"]["last_epoch"] == 1
    assert ours["scheduler"]["successor"]["last_epoch"] == ref["scheduler"]["successor"]["last_epoch"] == 1
    assert ours["scheduler"]["_last_lr"] == ref["scheduler"]["_last_lr"]
    p = torch.nn.Parameter(torch.zeros(4, 128))
    sgd = torch.optim.SGD([p], lr=0.1, momentum=0.9)
    sgd.load_state_dict(ours["optimizer"])  # what the reference's resume does
    t2 = _dummy_trainer(tmp_path, n_ctx=4, W=128, C=5)
    assert t2.resume_model_if_exist(str(tmp_path / "ours")) == 2
    assert t2.get_current_lr() == t.get_current_lr()


def test_checkpoint_layout_and_resume(tmp_path):
    """Dassl checkpoint format (torchtools.py:27-157, trainer.py:118-145): OUTPUT_DIR/<name>/
    model.pth.tar-<epoch> with keys state_dict/epoch/optimizer/scheduler/val_result plus a
    `checkpoint` pointer file; resume restores weights, scheduler and the start epoch."""
    import torch
    import torch.nn as nn
    from fsp_amd.engine.config import get_cfg_default
    from fsp_amd.engine.optim import build_optimizer, build_lr_scheduler
    from fsp_amd.engine.trainer import TrainerX

    class Learner(nn.Module):
        def __init__(self):
            super().__init__()
            self.ctx = nn.Parameter(torch.zeros(4, 8))
            self.register_buffer("token_prefix", torch.ones(3, 1, 8))

    class Dummy(TrainerX):
        def build_model(self):
            self.model = Learner()
            self.optim = build_optimizer(self.model, self.cfg.OPTIM)
            self.sched = build_lr_scheduler(self.optim, self.cfg.OPTIM)
            self.register_model("prompt_learner", self.model, self.optim, self.sched)

    cfg = get_cfg_default()
    cfg.OUTPUT_DIR = str(tmp_path)
    cfg.OPTIM.MAX_EPOCH = 5
    t = Dummy(cfg)
    with torch.no_grad():
        t.model.ctx.copy_(torch.arange(32.0).reshape(4, 8))
    t.update_lr()
    t.update_lr()
    lr = t.get_current_lr()
    t.save_model(2, str(tmp_path), val_result=0.5)
    d = tmp_path / "prompt_learner"
    assert (d / "checkpoint").read_text().strip() == "model.pth.tar-3"
    ck = torch.load(d / "model.pth.tar-3", map_location="cpu", weights_only=True)
    assert set(ck) == {"state_dict", "epoch", "optimizer", "scheduler", "val_result"}
    assert ck["epoch"] == 3 and ck["val_result"] == 0.5
    assert set(ck["state_dict"]) == {"ctx", "token_prefix"}
    t2 = Dummy(cfg)
    assert t2.resume_model_if_exist(str(tmp_path)) == 3
    assert torch.equal(t2.model.ctx, t.model.ctx)
    assert t2.get_current_lr() == lr
    with pytest.raises(KeyError):
        t2.register_model("prompt_learner", t2.model, None, None)


def test_best_val_final_model(tmp_path):
    """TEST.FINAL_MODEL "best_val" (Dassl trainer.py:402-443): a val test after every epoch,
    model-best.pth.tar written when the val result improves (val_result recorded), and the
    final test runs on the best-val weights loaded back by load_model."""
    from fsp_amd.engine import checkpoint as C
    rs = np.random.RandomState(3)
    batches = [{"img": torch.from_numpy(rs.randn(5, 3, 2, 2).astype(np.float32)),
                "label": torch.from_numpy(rs.randint(0, 3, 5))} for _ in range(2)]
    t = _dummy_trainer(tmp_path, batches)
    t.dm.val_loader = batches[:1]
    t.cfg.TEST.NO_TEST = False
    t.cfg.TEST.FINAL_MODEL = "best_val"
    vals = iter([10.0, 30.0, 20.0])
    tests = []
    orig_test = t.test

    def fake_test(split=None, return_pred=False):
        if split == "val":
            return next(vals)
        tests.append(t.learner.ctx.detach().clone())
        return orig_test(split, return_pred)
    t.test = fake_test
    t.run_epoch = lambda: t.learner.ctx.data.add_(1.0)  # epoch e leaves ctx == e + 1
    t.train(start_epoch=0, max_epoch=3)
    best = C.load_checkpoint(str(tmp_path / "prompt_learner" / "model-best.pth.tar"))
    assert best["epoch"] == 2 and best["val_result"] == 30.0  # the 2nd epoch's val was best
    assert float(best["state_dict"]["ctx"][0, 0]) == 2.0
    assert (tmp_path / "prompt_learner" / "model.pth.tar-3").exists()
    assert len(tests) == 1 and float(tests[0][0, 0]) == 2.0  # final test on the best-val weights


def test_resume_keeps_the_modules_own_keys(tmp_path):
    """A checkpoint holding more than the registered module (the reference's deep trainers
    register the whole CustomCLIP, frozen encoders included) resumes: extra keys dropped,
    the module's own keys required."""
    from fsp_amd.engine import checkpoint as C
    t = _dummy_trainer(tmp_path, n_ctx=4, W=8, C=3)
    sd = dict(t.learner.state_dict())
    sd = {k: v + 1 for k, v in sd.items()}
    sd["image_encoder.conv1.weight"] = torch.zeros(2, 2)
    C.save_checkpoint({"state_dict": sd, "epoch": 1, "optimizer": None, "scheduler": None, "val_result": None},
                      str(tmp_path / "ck" / "prompt_learner"))
    assert t.resume_model_if_exist(str(tmp_path / "ck")) == 1
    assert float(t.learner.ctx[0, 0]) == 1.0
    del sd["ctx"]
    C.save_checkpoint({"state_dict": sd, "epoch": 1, "optimizer": None, "scheduler": None, "val_result": None},
                      str(tmp_path / "ck2" / "prompt_learner"))
    with pytest.raises(RuntimeError, match="Missing key"):
        t.resume_model_if_exist(str(tmp_path / "ck2"))


def test_ln_fold_weights_split_contract(monkeypatch):
    """PREC fp32s LayerNorm fold tables (clip/model.py ln_fold_weights(split=True)): W' goes to
    clipk_split_pack as fp32 W diag(gamma), and s sums the value the split GEMM multiplies by,
    (hi + lo) / SPLIT_SCALE with hi = fp16(64 W'), lo = fp16(64 W' - hi) (clipk_split_pack), so the
    fold's mean term cancels against the operand actually used; c = b + W beta as the 16-bit form."""
    from fsp_amd import ops, _native as N
    from fsp_amd.clip import model as M
    seen = {}
    monkeypatch.setattr(ops, "split_pack", lambda w: seen.setdefault("w", w.clone()))
    g = torch.Generator().manual_seed(3)
    w = torch.randn(24, 64, generator=g) / 8
    w[0, :5] = torch.tensor([1e-9, -3e-7, 2.5e-5, 0.7, -1.3])  # tiny, subnormal-lo and large parts
    gamma = 1 + 0.2 * torch.randn(64, generator=g)
    beta = 0.1 * torch.randn(64, generator=g)
    b = 0.05 * torch.randn(24, generator=g)
    wp, s, c = M.ln_fold_weights(w, b, gamma, beta, torch.float32, "cpu", split=True)
    ref_wp = (w.double() * gamma.double()[None, :]).float()
    assert torch.equal(seen["w"], ref_wp) and wp is not None
    x = ref_wp * N.SPLIT_SCALE
    hi = x.half().float()
    lo = (x - hi).half().float()
    assert torch.equal(s, ((hi.double() + lo.double()) / N.SPLIT_SCALE).sum(1).float())
    assert torch.equal(c, (b.double() + w.double() @ beta.double()).float())
    # the packed value is W' to ~2^-22 relative: s is the fp32 row sum up to that
    assert torch.allclose(s.double(), ref_wp.double().sum(1), rtol=0, atol=1e-6 * float(ref_wp.abs().sum(1).max()))
    # out of the fp16 range at the split scale: no fold table (the encoder runs the LN passes)
    big = torch.full((2, 64), 2000.0)
    assert M.ln_fold_weights(big, torch.zeros(2), torch.ones(64), torch.zeros(64), torch.float32, "cpu",
                             split=True) is None
