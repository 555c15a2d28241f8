"""PREC fp32s on fp16-valued weights (CLIPK_F32S16, include/clipk.h).

The released CLIP checkpoints store fp16 weights (the reference loads them from the fp16
archive and copies them into its fp32 model: PromptSRC/clip/clip.py:154-180, model.py:699-701),
so clipk_split_pack's lo parts of such a weight are all zero and the hi(a) lo(b) product of the
split GEMM is exactly zero (a v_mfma whose products are all zero returns C unchanged:
tools/lab/mfma_zero.hip, profiles/r05w16/mfma_zero.txt). CLIPK_F32S16 skips it. The bar is
bitwise: every output equals the 3-MFMA form's (torch.equal), GEMM by GEMM and through the whole
CoCoOp step, and the step is within the fp32 gates of the oracle run on the same fp16-valued
weights (|d logit| <= 1e-3, gradients rel <= 1e-3). On every tile path: the 2- / 4-slot loop's
first 2-MFMA build was off by up to 5e-2 at 4k-8k rows -- an MFMA reading the split's
inline-asm writes too early (profiles/r05w16/hazard.txt) -- which these cases caught."""
import math
import os

import numpy as np
import pytest
import torch

from fsp_amd import ops, _native as N
from parity_util import run_native, rel_err

pytestmark = pytest.mark.gpu


def _w16(shape, g, scale):
    return (torch.randn(*shape, generator=g) * scale).half().float()


def test_split_lo_zero(dev):
    """clipk_split_lo_zero: 1 for an fp16-valued weight, 0 once one element is not."""
    g = torch.Generator(device="cpu").manual_seed(0)
    w = _w16((512, 2048), g, 0.03).to(dev)
    assert ops.split_lo_zero(ops.split_pack(w))
    w2 = w.clone()
    w2[511, 2047] += 2.0 ** -20
    assert not ops.split_lo_zero(ops.split_pack(w2))
    assert not ops.split_lo_zero(ops.split_pack(torch.randn(128, 64, generator=g).to(dev)))


@pytest.mark.parametrize("M", [300, 4600, 47160])
@pytest.mark.parametrize("Nn,K", [(512, 2048), (2048, 512), (1536, 512), (512, 512)])
def test_gemm_w16_vs_f32s(dev, M, Nn, K):
    """CLIPK_F32S16 == CLIPK_F32S bit for bit on an fp16-valued weight, every epilogue and the
    LayerNorm-statistics producer, on the small-M, 128x128 and 192x256 ping-pong tiles."""
    g = torch.Generator(device="cpu").manual_seed(M + Nn + K)
    a = torch.randn(M, K, generator=g).to(dev)
    b = _w16((Nn, K), g, 1 / math.sqrt(K)).to(dev)
    bias = torch.randn(Nn, generator=g).to(dev)
    res = torch.randn(M, Nn, generator=g).to(dev)
    aux = torch.randn(M, Nn, generator=g).to(dev)
    bp = ops.split_pack(b)
    assert ops.split_lo_zero(bp)
    cases = [(N.EPI_NONE, {}), (N.EPI_BIAS, {"bias": bias}), (N.EPI_BIAS_RES, {"bias": bias, "res": res}),
             (N.EPI_BIAS_QGELU, {"bias": bias, "want_out2": True}),
             (N.EPI_BIAS_QGELU | N.QGELU_DERIV, {"bias": bias, "want_out2": True}),
             (N.EPI_DQGELU, {"aux": aux}), (N.EPI_DQGELU | N.QGELU_DERIV, {"aux": aux})]
    for epi, kw in cases:
        o3 = ops.gemm(a, bp, epi, **kw)
        o2 = ops.gemm(a, bp, epi, w16=True, **kw)
        o3 = o3 if isinstance(o3, tuple) else (o3,)
        o2 = o2 if isinstance(o2, tuple) else (o2,)
        for x, y in zip(o2, o3):
            assert torch.equal(x, y), f"epi {epi:#x}: {int((x != y).sum())} outputs differ"
    # the same product to fp64: the split's fp32-class accuracy holds
    ref = a.double() @ b.double().t()
    o = ops.gemm(a, bp, N.EPI_NONE, w16=True)
    assert ((o.double() - ref).abs().max() / ref.abs().max()).item() <= 4e-6
    if Nn % 64 == 0 and M >= 16:
        st3 = torch.empty(M, Nn // 64, 2, device=dev)
        st2 = torch.empty_like(st3)
        y3 = ops.gemm_ln(a, bp, N.EPI_BIAS_RES, bias, stats=st3, res=res)
        y2 = ops.gemm_ln(a, bp, N.EPI_BIAS_RES, bias, stats=st2, res=res, w16=True)
        assert torch.equal(y2, y3) and torch.equal(st2, st3)


def test_w16_on_fp32_weights_is_the_rounded_weight(dev):
    """CLIPK_F32S16 on a weight with nonzero lo parts is a caller error the split_lo_zero check
    prevents (the encoders' split_mode): the lo part is then dropped, i.e. the product is that of
    the weight rounded to fp16 (SPLIT_SCALE * W to fp16)."""
    g = torch.Generator(device="cpu").manual_seed(7)
    a = torch.randn(4600, 512, generator=g).to(dev)  # N = 2048 at 4.6k rows: the ping-pong tiles
    b = (torch.randn(2048, 512, generator=g) * 0.04).to(dev)
    bp = ops.split_pack(b)
    assert not ops.split_lo_zero(bp)
    want = ops.gemm(a, ops.split_pack((b * N.SPLIT_SCALE).half().float() / N.SPLIT_SCALE), N.EPI_NONE)
    got = ops.gemm(a, bp, N.EPI_NONE, w16=True)
    assert torch.equal(got, want)


def _cocoop_c1000_b2(dev, fp16_values, monkeypatch, w16, fold=True):
    monkeypatch.setenv("FSP_SPLIT_W16", "1" if w16 else "0")
    monkeypatch.setenv("FSP_LN_FOLD", "1" if fold else "0")
    meta = {"arch": "ViT-B/16", "n_cls": 1000, "batch": 2, "n_ctx": 4, "ctx_init": "a photo of a", "focal": 0}
    return run_native(meta, {"ctx0": None, "tokenized": None}, "fp32s", cocoop=True, dev=str(dev),
                      fp16_values=fp16_values)


def test_cocoop_headline_w16_bitwise(dev, monkeypatch):
    """The headline shape (CoCoOp ViT-B/16, C = 1000, B = 2, packed rows) in PREC fp32s on
    fp16-valued weights, without the LayerNorm fold (whose mode-2 form, gamma on A, rounds
    differently from mode 1's W diag(gamma): test_cocoop_headline_w16_vs_oracle): the encoders pick
    split mode 2 (CLIPK_F32S16 for every GEMM), and logits, loss, image features and every gradient
    are bitwise those of split mode 1 (FSP_SPLIT_W16=0). On fp32-valued weights mode 1 stays."""
    out2 = _cocoop_c1000_b2(dev, True, monkeypatch, True, fold=False)
    out1 = _cocoop_c1000_b2(dev, True, monkeypatch, False, fold=False)
    assert out2["split_modes"] == (2, 2), out2["split_modes"]
    assert out1["split_modes"] == (1, 1), out1["split_modes"]
    for k in out1:
        if k.startswith("grad_") or k in ("image_features", "logits", "ctx_after_step"):
            np.testing.assert_array_equal(out2[k], out1[k], err_msg=k)
    assert out2["loss"] == out1["loss"]
    mixed = _cocoop_c1000_b2(dev, False, monkeypatch, True)
    assert mixed["split_modes"] == (1, 1)


def test_cocoop_headline_w16_vs_oracle(dev, monkeypatch):
    """The same step with the LayerNorm fold (mode 2: gamma on A, every GEMM CLIPK_F32S16) against
    the CPU oracle run on the same fp16-valued weights: the fp32 gates."""
    from test_parity_gpu import _cocoop_oracle
    ref = _cocoop_oracle("ViT-B/16", 1000, 2, fp16_values=True)
    out = _cocoop_c1000_b2(dev, True, monkeypatch, True)
    assert out["split_modes"] == (2, 2)
    np.testing.assert_array_equal(out["ctx0"], ref["ctx0"])
    assert float(np.abs(out["logits"] - ref["logits"]).max()) <= 1e-3
    assert abs(out["loss"] - ref["loss"]) <= 1e-4 * max(1.0, abs(ref["loss"]))
    for g in [k for k in ref if k.startswith("grad_")]:
        assert rel_err(out[g], ref[g]) <= 1e-3, g
