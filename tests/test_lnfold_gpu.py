"""LayerNorm folded into the text GEMMs (clipk_gemm_ln / clipk_ln_stats_merge /
clipk_encoder_set_ln_fold) vs PyTorch fp32/fp64 references of the same ops.

The fold rewrites LN(x) W^T + b (PromptSRC/clip/model.py:153-159 feeding 171-177 / 185-188)
as rstd * (x W'^T - mean * s) + c, W' = W diag(gamma): the producer GEMM writes per-row
statistics partials of the residual stream it stores, and the consumer GEMM reads x itself.
Bars: the statistics match torch on the stored (rounded) values to fp32 rounding; the folded
GEMM is within the dtype's tolerance of the fp64 reference and no further from it than the
un-fused path (LayerNorm pass -> 16-bit -> GEMM) by more than a small margin. PREC fp32s (fp32
stream, split-packed W'): the same at fp32-class bars."""
import math
import os

import pytest
import torch
import torch.nn.functional as F

from fsp_amd import ops, _native as N
from fsp_amd.clip import model as M, synth
from fsp_amd.trainers.prompt_base import TextShape

pytestmark = pytest.mark.gpu

TOL = {torch.float16: 1e-2, torch.bfloat16: 3e-2}


def partials(x):
    """The producer's statistics partials of x (what an EPI_BIAS_RES clipk_gemm_ln writes)."""
    xg = x.double().reshape(x.shape[0], -1, 64)
    return torch.stack([xg.sum(-1), ((xg - xg.mean(-1, keepdim=True)) ** 2).sum(-1)], -1).float().contiguous()


def _rel(out, ref):
    return ((out.double() - ref.double()).abs().max() / (ref.double().abs().max() + 1e-30)).item()


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("Mr,Nn,K", [(47160, 512, 2048), (8000, 512, 512), (300, 768, 512), (20000, 768, 3072),
                                     (1, 512, 512)])
def test_gemm_ln_stats(dev, dtype, Mr, Nn, K):
    g = torch.Generator(device="cpu").manual_seed(Mr + Nn + K)
    a = torch.randn(Mr, K, generator=g).to(dev, dtype)
    b = (torch.randn(Nn, K, generator=g) / math.sqrt(K)).to(dev, dtype)
    bias = (0.1 * torch.randn(Nn, generator=g)).to(dev)
    # residual stream with a per-row offset and an outlier column (CLIP's large-magnitude dims)
    res = torch.randn(Mr, Nn, generator=g) + 3.0 * torch.randn(Mr, 1, generator=g)
    res[:, 7] *= 40.0
    res = res.to(dev, dtype)
    stats = torch.full((Mr, Nn // 64, 2), float("nan"), device=dev)
    out = ops.gemm_ln(a, b, N.EPI_BIAS_RES, bias, stats, res=res)
    plain = ops.gemm(a, b, N.EPI_BIAS_RES, dtype, bias=bias, res=res)
    assert torch.equal(out, plain), "stats epilogue changed the stored output"
    mean, rstd, rnb = ops.ln_stats_merge(stats, Nn)
    assert torch.equal(rnb[:, 0], rstd) and torch.equal(rnb[:, 1], -rstd * mean)
    x = out.double()
    mu = x.mean(1)
    var = x.var(1, unbiased=False)
    assert ((mean.double() - mu).abs() <= 1e-5 * (x.abs().amax(1) + 1)).all()
    assert ((rstd.double() * torch.sqrt(var + 1e-5) - 1).abs().max().item()) <= 2e-5


@pytest.mark.parametrize("Wd", [128, 512, 768, 1024])
@pytest.mark.parametrize("Mr", [1, 31, 33, 4097, 150001])
def test_ln_stats_merge_widths(dev, Wd, Mr):
    """clipk_ln_stats_merge alone: 8-lane (width <= 512) and 16-lane row groups, 4 rows per lane
    group, ragged row counts; vs the fp64 statistics of x, and
    bitwise-equal reruns."""
    g = torch.Generator(device="cpu").manual_seed(Mr + Wd)
    x = torch.randn(Mr, Wd, generator=g) + 3.0 * torch.randn(Mr, 1, generator=g)
    x[:, 3] *= 25.0
    st = partials(x).to(dev)
    mean, rstd, rnb = ops.ln_stats_merge(st, Wd)
    m2, r2, n2 = ops.ln_stats_merge(st, Wd)
    assert torch.equal(mean, m2) and torch.equal(rstd, r2) and torch.equal(rnb, n2)
    assert torch.equal(rnb[:, 0], rstd) and torch.equal(rnb[:, 1], -rstd * mean)
    xd = x.double().to(dev)
    mu, var = xd.mean(1), xd.var(1, unbiased=False)
    assert ((mean.double() - mu).abs() <= 1e-5 * (xd.abs().amax(1) + 1)).all()
    assert ((rstd.double() * torch.sqrt(var + 1e-5) - 1).abs().max().item()) <= 2e-5


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("epi", [N.EPI_BIAS, N.EPI_BIAS_QGELU])
@pytest.mark.parametrize("Mr,Wd,Nn", [(47160, 512, 1536), (47160, 512, 2048), (8000, 512, 2048), (300, 768, 2304),
                                      (3, 512, 1536)])
def test_gemm_ln_fold(dev, dtype, epi, Mr, Wd, Nn):
    g = torch.Generator(device="cpu").manual_seed(Mr * 3 + Wd + Nn + epi)
    x = torch.randn(Mr, Wd, generator=g) + 2.0 * torch.randn(Mr, 1, generator=g)
    x[:, 5] *= 30.0
    x = x.to(dev, dtype)
    gamma = (1.0 + 0.2 * torch.randn(Wd, generator=g)).to(dev)
    beta = (0.1 * torch.randn(Wd, generator=g)).to(dev)
    w = (torch.randn(Nn, Wd, generator=g) / math.sqrt(Wd)).to(dev)
    bias = (0.05 * torch.randn(Nn, generator=g)).to(dev)
    wp, s, c = M.ln_fold_weights(w, bias, gamma, beta, dtype, dev)
    xd = x.double()
    ref = F.layer_norm(xd, (Wd,), gamma.double(), beta.double(), eps=1e-5) @ w.double().t() + bias.double()
    if epi == N.EPI_BIAS_QGELU:
        ref_g = ref * torch.sigmoid(1.702 * ref)
    # the un-fused path the fold replaces: LayerNorm pass -> 16-bit -> GEMM with W
    xn = ops.layernorm(x, gamma, beta, out_dtype=dtype)
    wq = w.to(dtype)
    mean, rstd, rnb = ops.ln_stats_merge(partials(x), Wd)
    if epi == N.EPI_BIAS:
        out = ops.gemm_ln(x, wp, epi, c, colsum=s, rnb=rnb)
        unf = ops.gemm(xn, wq, N.EPI_BIAS, dtype, bias=bias)
        e_fold, e_unf = _rel(out, ref), _rel(unf, ref)
    else:
        out, h = ops.gemm_ln(x, wp, epi, c, colsum=s, rnb=rnb, want_out2=True)
        unf, uh = ops.gemm(xn, wq, N.EPI_BIAS_QGELU, dtype, bias=bias, want_out2=True)
        e_fold, e_unf = max(_rel(out, ref_g), _rel(h, ref)), max(_rel(unf, ref_g), _rel(uh, ref))
    mu, var = xd.mean(1), xd.var(1, unbiased=False)
    assert ((mean.double() - mu).abs() <= 1e-5 * (xd.abs().amax(1) + 1)).all()
    assert ((rstd.double() * torch.sqrt(var + 1e-5) - 1).abs().max().item()) <= 2e-5
    assert e_fold <= TOL[dtype], f"fold rel err {e_fold:.3e}"
    assert e_fold <= 1.5 * e_unf + 2e-3, f"fold {e_fold:.3e} vs un-fused {e_unf:.3e}"
    if epi == N.EPI_BIAS_QGELU and Mr >= 8000:
        # training's fold form (CLIPK_QGELU_DERIV): out2 = quickgelu'(pre-activation)
        og, d = ops.gemm_ln(x, wp, epi | N.QGELU_DERIV, c, colsum=s, rnb=rnb, want_out2=True)
        sg = torch.sigmoid(1.702 * ref)
        assert torch.equal(og, out), "the QuickGELU output does not depend on what out2 holds"
        assert _rel(d, sg * (1 + 1.702 * ref * (1 - sg))) <= TOL[dtype]


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("epi", [N.EPI_BIAS, N.EPI_BIAS_QGELU, N.EPI_BIAS_QGELU | N.QGELU_DERIV])
@pytest.mark.parametrize("Mr,Nn,fused", [(5895, 1536, True), (5895, 2048, True), (5000, 2048, True),
                                         (47160, 1536, False), (3000, 2048, False), (1, 1536, False)])
def test_gemm_ln_merge_equals_two_launches(dev, dtype, epi, Mr, Nn, fused):
    """clipk_gemm_ln_merge (the statistics merge inside the folding GEMM: the batch-1 text shapes,
    5.9k rows on 192-row tiles) against clipk_ln_stats_merge + clipk_gemm_ln: every output
    bitwise equal (out, out2, mean, rstd, rnb), ragged last row block included; the shapes the
    library does not fuse take the two launches themselves."""
    Wd = 512
    assert N.load().clipk_gemm_ln_merge_fused(N.F16 if dtype == torch.float16 else N.BF16, Mr, Nn, Wd) == int(fused)
    g = torch.Generator(device="cpu").manual_seed(Mr + Nn + epi)
    x = torch.randn(Mr, Wd, generator=g) + 2.0 * torch.randn(Mr, 1, generator=g)
    x[:, 5] *= 30.0
    x = x.to(dev, dtype)
    gamma = (1.0 + 0.2 * torch.randn(Wd, generator=g)).to(dev)
    beta = (0.1 * torch.randn(Wd, generator=g)).to(dev)
    w = (torch.randn(Nn, Wd, generator=g) / math.sqrt(Wd)).to(dev)
    bias = (0.05 * torch.randn(Nn, generator=g)).to(dev)
    wp, s, c = M.ln_fold_weights(w, bias, gamma, beta, dtype, dev)
    st = partials(x)
    two = epi != N.EPI_BIAS
    mean, rstd, rnb = ops.ln_stats_merge(st, Wd)
    ref = ops.gemm_ln(x, wp, epi, c, colsum=s, rnb=rnb, want_out2=two)
    ref = ref if two else (ref,)
    got = ops.gemm_ln_merge(x, wp, epi, c, st, s, want_out2=two)
    for nm, u, v in zip(("out", "out2", "mean", "rstd", "rnb") if two else ("out", "mean", "rstd", "rnb"),
                        got, tuple(ref) + (mean, rstd, rnb)):
        assert torch.equal(u, v), f"{nm} differs from the two-launch form"


def test_gemm_ln_merge_empty_and_negative_rows(dev, monkeypatch):
    """clipk_gemm_ln_merge with M = 0 is a no-op (CLIPK_OK) and M < 0 a shape error, also when
    the fused form is forced (the fused path launched a zero-block grid)."""
    monkeypatch.setenv("CLIPK_GEMM_CFG", "6")
    lib = N.load()
    x = torch.zeros(8, 512, device=dev, dtype=torch.float16)
    w = torch.zeros(512, 512, device=dev, dtype=torch.float16)
    f = torch.zeros(4096, device=dev)
    for m, want in ((0, 0), (-3, -2)):
        rc = lib.clipk_gemm_ln_merge(N.F16, N.EPI_BIAS, m, 512, 512, ops._p(x), 512, ops._p(w), 512, ops._p(f),
                                     ops._p(x), 512, None, ops._p(f), ops._p(f), ops._p(f), ops._p(f), ops._p(f),
                                     ops._stream())
        assert rc == want, (m, rc)


@pytest.mark.parametrize("Mr,Nn,K", [(47160, 512, 2048), (8000, 512, 512), (300, 512, 2048), (1, 512, 512)])
def test_gemm_ln_stats_split(dev, Mr, Nn, K):
    """PREC fp32s statistics producer (fp32 out, 16 lanes per 64-column group): the stored output
    is bitwise the plain split GEMM's, the partials merge to the fp64 statistics of it."""
    g = torch.Generator(device="cpu").manual_seed(Mr + Nn + K + 1)
    a = torch.randn(Mr, K, generator=g).to(dev)
    b = ops.split_pack((torch.randn(Nn, K, generator=g) / math.sqrt(K)).to(dev))
    bias = (0.1 * torch.randn(Nn, generator=g)).to(dev)
    res = torch.randn(Mr, Nn, generator=g) + 3.0 * torch.randn(Mr, 1, generator=g)
    res[:, 7] *= 40.0
    res = res.to(dev)
    stats = torch.full((Mr, Nn // 64, 2), float("nan"), device=dev)
    out = ops.gemm_ln(a, b, N.EPI_BIAS_RES, bias, stats, res=res)
    plain = ops.gemm(a, b, N.EPI_BIAS_RES, torch.float32, bias=bias, res=res)
    assert torch.equal(out, plain), "stats epilogue changed the stored output"
    ref = partials(out)
    assert torch.allclose(stats[..., 0], ref[..., 0], rtol=0, atol=1e-4 * float(out.abs().max()))
    assert ((stats[..., 1] - ref[..., 1]).abs() <= 1e-5 * ref[..., 1] + 1e-3).all()
    mean, rstd, _ = ops.ln_stats_merge(stats, Nn)
    x = out.double()
    assert ((mean.double() - x.mean(1)).abs() <= 1e-6 * (x.abs().amax(1) + 1)).all()
    assert ((rstd.double() * torch.sqrt(x.var(1, unbiased=False) + 1e-5) - 1).abs().max().item()) <= 2e-6


@pytest.mark.parametrize("epi", [N.EPI_BIAS, N.EPI_BIAS_QGELU])
@pytest.mark.parametrize("Mr,Wd,Nn", [(47160, 512, 1536), (8000, 512, 2048), (300, 512, 2048), (3, 512, 1536)])
def test_gemm_ln_fold_split(dev, epi, Mr, Wd, Nn):
    """PREC fp32s fold (fp32 x, split-packed W'): within fp32-class tolerance of the fp64
    LayerNorm -> Linear, and no further from it than the un-fused fp32s path (fp32 LayerNorm
    pass -> split GEMM with W) by more than fp32 rounding."""
    g = torch.Generator(device="cpu").manual_seed(Mr * 5 + Wd + Nn + epi)
    x = torch.randn(Mr, Wd, generator=g) + 2.0 * torch.randn(Mr, 1, generator=g)
    x[:, 5] *= 30.0
    x = x.to(dev)
    gamma = (1.0 + 0.2 * torch.randn(Wd, generator=g)).to(dev)
    beta = (0.1 * torch.randn(Wd, generator=g)).to(dev)
    w = (torch.randn(Nn, Wd, generator=g) / math.sqrt(Wd)).to(dev)
    bias = (0.05 * torch.randn(Nn, generator=g)).to(dev)
    wp, s, c = M.ln_fold_weights(w.cpu(), bias.cpu(), gamma.cpu(), beta.cpu(), torch.float32, dev, split=True)
    xd = x.double()
    ref = F.layer_norm(xd, (Wd,), gamma.double(), beta.double(), eps=1e-5) @ w.double().t() + bias.double()
    xn = ops.layernorm(x, gamma, beta, out_dtype=torch.float32)
    wq = ops.split_pack(w)
    _, _, rnb = ops.ln_stats_merge(partials(x), Wd)
    if epi == N.EPI_BIAS:
        out = ops.gemm_ln(x, wp, epi, c, colsum=s, rnb=rnb)
        unf = ops.gemm(xn, wq, N.EPI_BIAS, torch.float32, bias=bias)
        e_fold, e_unf = _rel(out, ref), _rel(unf, ref)
    else:
        ref_g = ref * torch.sigmoid(1.702 * ref)
        out, d = ops.gemm_ln(x, wp, epi | N.QGELU_DERIV, c, colsum=s, rnb=rnb, want_out2=True)
        unf = ops.gemm(xn, wq, N.EPI_BIAS_QGELU, torch.float32, bias=bias)
        sg = torch.sigmoid(1.702 * ref)
        e_fold = max(_rel(out, ref_g), _rel(d, sg * (1 + 1.702 * ref * (1 - sg))))
        e_unf = _rel(unf, ref_g)
    # the fold's rstd * (x W'^T) - rstd * mean * s cancels: its rounding scales with the row's
    # rms / std = sqrt(1 + mean^2 / var) (up to ~5 for these rows: offsets 2 N(0, 1), std ~1.7),
    # the un-fused path's (which rounds the normalised row) does not
    mu, var = xd.mean(1), xd.var(1, unbiased=False)
    amp = float(torch.sqrt(1 + mu * mu / var).max())
    assert e_fold <= 2e-5, f"fold rel err {e_fold:.3e}"
    assert e_fold <= 2.0 * amp * e_unf + 2e-6, f"fold {e_fold:.3e} vs un-fused {e_unf:.3e} (amp {amp:.2f})"


@pytest.mark.parametrize("w16", [False, True])
@pytest.mark.parametrize("epi", [N.EPI_BIAS, N.EPI_BIAS_QGELU])
@pytest.mark.parametrize("Mr,Wd,Nn", [(47160, 512, 1536), (8000, 512, 2048), (300, 512, 2048), (3, 512, 1536),
                                      (5000, 768, 2304)])
def test_gemm_ln_gamma_split(dev, epi, Mr, Wd, Nn, w16):
    """PREC fp32s fold with the LayerNorm weight on A (clipk_gemm_ln_gamma: B = W itself, x * gamma
    in fp32 before the split), on an fp16-valued W (split mode 2's weights; w16: CLIPK_F32S16,
    bitwise the 3-MFMA form on the tiles it runs on): the gates of test_gemm_ln_fold_split against
    the fp64 LayerNorm -> Linear, on every tile path (ping-pong, 128x128, 64x128)."""
    g = torch.Generator(device="cpu").manual_seed(Mr * 7 + Wd + Nn + epi)
    x = torch.randn(Mr, Wd, generator=g) + 2.0 * torch.randn(Mr, 1, generator=g)
    x[:, 5] *= 30.0
    x = x.to(dev)
    gamma = (1.0 + 0.2 * torch.randn(Wd, generator=g)).to(dev)
    beta = (0.1 * torch.randn(Wd, generator=g)).to(dev)
    w = (torch.randn(Nn, Wd, generator=g) / math.sqrt(Wd)).half().float().to(dev)
    bias = (0.05 * torch.randn(Nn, generator=g)).to(dev)
    wh, s, c = M.ln_fold_weights(w.cpu(), bias.cpu(), gamma.cpu(), beta.cpu(), torch.float32, dev, split=True,
                                 gamma_on_a=True)
    assert wh.dtype == torch.float16  # mode 2's compact weight (ops.split_hi16)
    wpk = ops.split_pack(w)  # the packed form (CLIPK_F32S, 3 MFMAs per product)
    assert ops.split_lo_zero(wpk)
    assert torch.equal(wh, ops.split_hi16(wpk))
    wp = wh if w16 else wpk
    xd = x.double()
    ref = F.layer_norm(xd, (Wd,), gamma.double(), beta.double(), eps=1e-5) @ w.double().t() + bias.double()
    xn = ops.layernorm(x, gamma, beta, out_dtype=torch.float32)
    _, _, rnb = ops.ln_stats_merge(partials(x), Wd)
    if epi == N.EPI_BIAS:
        out = ops.gemm_ln_gamma(x, wp, epi, c, s, rnb, gamma)
        unf = ops.gemm(xn, wp, N.EPI_BIAS, torch.float32, bias=bias)
        e_fold, e_unf = _rel(out, ref), _rel(unf, ref)
    else:
        ref_g = ref * torch.sigmoid(1.702 * ref)
        out, d = ops.gemm_ln_gamma(x, wp, epi | N.QGELU_DERIV, c, s, rnb, gamma, want_out2=True)
        unf = ops.gemm(xn, wp, N.EPI_BIAS_QGELU, torch.float32, bias=bias)
        sg = torch.sigmoid(1.702 * ref)
        e_fold = max(_rel(out, ref_g), _rel(d, sg * (1 + 1.702 * ref * (1 - sg))))
        e_unf = _rel(unf, ref_g)
    if w16:  # the 2-MFMA form on the compact weight equals the 3-MFMA one on the packed weight
        o3 = ops.gemm_ln_gamma(x, wpk, epi, c, s, rnb, gamma)
        o2 = out if epi == N.EPI_BIAS else ops.gemm_ln_gamma(x, wh, epi, c, s, rnb, gamma)
        assert torch.equal(o2, o3)
    mu, var = xd.mean(1), xd.var(1, unbiased=False)
    amp = float(torch.sqrt(1 + mu * mu / var).max())
    print(f"gamma fold {Mr}x{Nn}x{Wd} w16={w16}: {e_fold:.2e} (un-fused {e_unf:.2e}, amp {amp:.2f})")
    assert e_fold <= 2e-5, f"fold rel err {e_fold:.3e}"
    assert e_fold <= 2.0 * amp * e_unf + 2e-6, f"fold {e_fold:.3e} vs un-fused {e_unf:.3e} (amp {amp:.2f})"


def _encoder_pair(arch, prec, dev):
    sd = synth.make_state_dict(arch, seed=0)
    a = synth.ARCHS[arch]
    os.environ["FSP_LN_FOLD"] = "0"
    try:
        off = M.TextEncoderCore(sd, a, prec, dev)
    finally:
        os.environ.pop("FSP_LN_FOLD", None)
    on = M.TextEncoderCore(sd, a, prec, dev)
    ref = M.TextEncoderCore(sd, a, "fp32", dev)
    return a, on, off, ref


@pytest.mark.parametrize("prec", ["fp16", "bf16", "amp", "fp32s"])
def test_text_encoder_fold_on_off(dev, prec):
    """Whole text encoder (12 layers, plain layout, EOT-last layer): the folded encoder's
    features and input gradient against the fp32 encoder, no worse than the un-fused one."""
    a, on, off, ref = _encoder_pair("ViT-B/16", prec, dev)
    nseq, L = 64, 11
    g = torch.Generator(device="cpu").manual_seed(5)
    x0 = (0.3 * torch.randn(nseq * L, a.transformer_width, generator=g)).to(dev)
    eot = (torch.arange(nseq) * L + (3 + torch.arange(nseq) % 8)).to(torch.int32).to(dev)
    shape = TextShape(eot, nseq=nseq, L=L)
    dtxt = torch.randn(nseq, a.embed_dim, generator=g).to(dev)
    res = {}
    for nm, core in (("on", on), ("off", off), ("ref", ref)):
        txt, saved = core.forward(x0, shape, save=True)
        dx0 = core.backward(dtxt, shape, saved)
        res[nm] = (txt.double(), dx0.double())
    def cos(u, v):
        return (1 - (u * v).sum() / (u.norm() * v.norm())).item()
    # only the rows that reach an EOT row carry a gradient
    live = torch.zeros(nseq * L, dtype=torch.bool, device=dev)
    for s in range(nseq):
        live[s * L:int(eot[s]) + 1] = True
    for i, nm in ((0, "txt"), (1, "dx0")):
        r = res["ref"][i] if i == 0 else res["ref"][i][live]
        e_on = cos((res["on"][i] if i == 0 else res["on"][i][live]).flatten(), r.flatten())
        e_off = cos((res["off"][i] if i == 0 else res["off"][i][live]).flatten(), r.flatten())
        bar = {"bf16": 5e-3, "fp32s": 1e-9}.get(prec, 1e-3)
        assert e_on <= bar, f"{nm}: fold 1-cos {e_on:.3e}"
        assert e_on <= 2.0 * e_off + (1e-11 if prec == "fp32s" else 1e-5), \
            f"{nm}: fold {e_on:.3e} vs un-fused {e_off:.3e}"
        if prec == "fp32s":  # fp32-class: the features themselves, not only their direction
            ro = (res["on"][i] if i == 0 else res["on"][i][live])
            assert _rel(ro, r) <= 1e-4, f"{nm}: fold rel err {_rel(ro, r):.3e}"
