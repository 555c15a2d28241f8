"""PREC fp32s on fp16-valued weights (CLIPK_F32S16, include/clipk.h).

The released CLIP checkpoints store fp16 weights (the reference loads them from the fp16
archive and copies them into its fp32 model: PromptSRC/clip/clip.py:154-180, model.py:699-701),
so clipk_split_pack's lo parts of such a weight are all zero and the hi(a) lo(b) product of the
split GEMM is exactly zero (a v_mfma whose products are all zero returns C unchanged:
tools/lab/mfma_zero.hip, profiles/r05w16/mfma_zero.txt). CLIPK_F32S16 skips it and takes B in
its compact form (clipk_split_hi16: fp16 SPLIT_SCALE * W, 2 B per element instead of the packed
4), so its K loop stages B's rows at half the bytes. The bar is
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
from fsp_amd.clip import model as M_
from parity_util import run_native, rel_err

pytestmark = pytest.mark.gpu


def _w16(shape, g, scale):
    return (torch.randn(*shape, generator=g) * scale).half().float()


def test_split_lo_zero(dev):
    """clipk_split_lo_zero: 1 for an fp16-valued weight, 0 once one element is not; split_hi16
    compacts the former (SPLIT_SCALE * W exactly in fp16) and refuses the latter (CLIPK_ERANGE)."""
    g = torch.Generator(device="cpu").manual_seed(0)
    w = _w16((512, 2048), g, 0.03).to(dev)
    bp = ops.split_pack(w)
    assert ops.split_lo_zero(bp)
    wh = ops.split_hi16(bp)
    assert wh.dtype == torch.float16 and wh.shape == w.shape
    assert torch.equal(wh.float(), w * N.SPLIT_SCALE)
    w2 = w.clone()
    w2[511, 2047] += 2.0 ** -20
    bp2 = ops.split_pack(w2)
    assert not ops.split_lo_zero(bp2)
    out = torch.empty(512, 2048, dtype=torch.float16, device=dev)
    lib = N.load()
    assert lib.clipk_split_hi16(512, 2048, ops._p(bp2), ops._p(out), ops._stream()) == -5  # CLIPK_ERANGE
    with pytest.raises(N.ClipkError):
        ops.split_hi16(bp2)
    assert not ops.split_lo_zero(ops.split_pack(torch.randn(128, 64, generator=g).to(dev)))


def test_split_checks_report_errors_not_answers(dev):
    """The weight checks report an argument error as a negative status and leave the answer
    untouched: a failed check is never read as 'fp16-valued' (a positive HIP error
    code from clipk_split_lo_zero used to equal its 'all lo parts zero' answer)."""
    import ctypes
    lib = N.load()
    res = ctypes.c_int(7)
    assert lib.clipk_split_lo_zero(128, 64, None, ctypes.byref(res), ops._stream()) < 0
    assert lib.clipk_split_lo_zero(128, 60, ops._p(torch.zeros(128, 64, dtype=torch.int32, device=dev)),
                                   ctypes.byref(res), ops._stream()) < 0
    assert res.value == 7
    ok = torch.zeros(128, 64, dtype=torch.int32, device=dev)
    assert lib.clipk_split_lo_zero(128, 64, ops._p(ok), None, ops._stream()) < 0
    assert lib.clipk_split_lo_zero(128, 64, ops._p(ok), ctypes.byref(res), ops._stream()) == 0
    assert res.value == 1
    # two threads checking different weights at once each get their own answer (per-call flags)
    import threading
    bad = ops.split_pack(torch.randn(256, 512, device=dev))
    good = ops.split_pack(torch.randn(256, 512, device=dev).half().float())
    answers = {}

    def run(name, t):
        with torch.cuda.stream(torch.cuda.Stream(dev)):
            answers[name] = [ops.split_lo_zero(t) for _ in range(20)]
    th = [threading.Thread(target=run, args=(n, t)) for n, t in (("bad", bad), ("good", good))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert answers == {"bad": [False] * 20, "good": [True] * 20}


@pytest.mark.parametrize("M", [300, 4600, 8000, 47160])
@pytest.mark.parametrize("Nn,K", [(512, 2048), (2048, 512), (1536, 512), (512, 512)])
def test_gemm_w16_vs_f32s(dev, M, Nn, K):
    """CLIPK_F32S16 on the compact weight == CLIPK_F32S on the packed weight bit for bit (an
    fp16-valued weight), every epilogue and the LayerNorm-statistics producer, on the small-M,
    128x128 and 192x256 ping-pong tiles."""
    g = torch.Generator(device="cpu").manual_seed(M + Nn + K)
    a = torch.randn(M, K, generator=g).to(dev)
    b = _w16((Nn, K), g, 1 / math.sqrt(K)).to(dev)
    bias = torch.randn(Nn, generator=g).to(dev)
    res = torch.randn(M, Nn, generator=g).to(dev)
    aux = torch.randn(M, Nn, generator=g).to(dev)
    bp = ops.split_pack(b)
    assert ops.split_lo_zero(bp)
    bh = ops.split_hi16(bp)
    cases = [(N.EPI_NONE, {}), (N.EPI_BIAS, {"bias": bias}), (N.EPI_BIAS_RES, {"bias": bias, "res": res}),
             (N.EPI_BIAS_QGELU, {"bias": bias, "want_out2": True}),
             (N.EPI_BIAS_QGELU | N.QGELU_DERIV, {"bias": bias, "want_out2": True}),
             (N.EPI_DQGELU, {"aux": aux}), (N.EPI_DQGELU | N.QGELU_DERIV, {"aux": aux})]
    for epi, kw in cases:
        o3 = ops.gemm(a, bp, epi, **kw)
        o2 = ops.gemm(a, bh, epi, **kw)
        o3 = o3 if isinstance(o3, tuple) else (o3,)
        o2 = o2 if isinstance(o2, tuple) else (o2,)
        for x, y in zip(o2, o3):
            assert torch.equal(x, y), f"epi {epi:#x}: {int((x != y).sum())} outputs differ"
    # the same product to fp64: the split's fp32-class accuracy holds
    ref = a.double() @ b.double().t()
    o = ops.gemm(a, bh, N.EPI_NONE)
    assert ((o.double() - ref).abs().max() / ref.abs().max()).item() <= 4e-6
    if Nn % 64 == 0 and M >= 16:
        st3 = torch.empty(M, Nn // 64, 2, device=dev)
        st2 = torch.empty_like(st3)
        y3 = ops.gemm_ln(a, bp, N.EPI_BIAS_RES, bias, stats=st3, res=res)
        y2 = ops.gemm_ln(a, bh, N.EPI_BIAS_RES, bias, stats=st2, res=res)
        assert torch.equal(y2, y3) and torch.equal(st2, st3)
    if M <= 8000:  # split-K slices (the ViT's small-M path) on the compact weight
        sk = ops.gemm_splitk(a, bh, N.EPI_NONE, splits=2) if K >= 512 else None
        if sk is not None:
            assert torch.equal(sk, ops.gemm_splitk(a, bp, N.EPI_NONE, splits=2))


def test_w16_refuses_fp32_weights(dev):
    """A weight with nonzero lo parts has no compact form: split_hi16 refuses it, so CLIPK_F32S16
    can never drop a weight's lo part (the encoders pick split mode 2 only when every weight passes
    split_lo_zero, and then compact each one through split_hi16, which checks again)."""
    g = torch.Generator(device="cpu").manual_seed(7)
    b = (torch.randn(2048, 512, generator=g) * 0.04).to(dev)
    bp = ops.split_pack(b)
    assert not ops.split_lo_zero(bp)
    with pytest.raises(N.ClipkError):
        ops.split_hi16(bp)


def test_encoder_split_mode_is_fixed(dev):
    """clipk_encoder_set_split: the mode names the tables' format, so it cannot change once set or
    under a LayerNorm fold (a mode change after set_ln_fold applied gamma twice or
    dropped it)."""
    from fsp_amd.clip import synth, model as M
    sd = synth.make_state_dict("tiny4", seed=0)
    core = M.TextEncoderCore(sd, synth.ARCHS["tiny4"], "fp32s", dev)
    lib = N.load()
    mode = core.split_mode
    assert mode in (1, 2)
    assert lib.clipk_encoder_set_split(core.handle, mode) == 0        # idempotent
    assert lib.clipk_encoder_set_split(core.handle, 3 - mode) == -1   # CLIPK_EINVAL
    assert lib.clipk_encoder_set_split(core.handle, 0) == -1


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


def split_form(x):
    """The pre-split operand form of fp32 x [M, K] (include/clipk.h CLIPK_OUT_SPLIT): per 8
    consecutive k, 8 fp16 hi = fp16(x) then 8 fp16 lo = fp16(x - hi), viewed as fp32 [M, K]."""
    M, K = x.shape
    hi = x.half()
    lo = (x - hi.float()).half()  # x - hi is exact in fp32
    t = torch.stack([hi.view(M, K // 8, 8), lo.view(M, K // 8, 8)], 2)
    return t.reshape(M, 2 * K).view(torch.float32)


@pytest.mark.parametrize("M", [300, 4600, 8000, 47160])
@pytest.mark.parametrize("mode", [1, 2])
def test_presplit_handoffs_bitwise(dev, M, mode):
    """The MLP's pre-split hand-offs (CLIPK_OUT_SPLIT producers, CLIPK_A_SPLIT consumers) are
    bitwise the fp32 hand-offs: c_fc (plain, W'-fold, gamma-fold) -> c_proj (plain and as the
    statistics producer), dgelu (saved derivative) -> fc_dx, on every tile path (M 300: 64x128,
    4,600 / 8,000: 128x128, 47,160: the 192x256 ping-pong tiles)."""
    W = 512
    g = torch.Generator(device="cpu").manual_seed(M + mode)
    x = (torch.randn(M, W, generator=g) + 0.5 * torch.randn(M, 1, generator=g)).to(dev)
    wfc = _w16((4 * W, W), g, 1 / math.sqrt(W)).to(dev)
    wpj = _w16((W, 4 * W), g, 1 / math.sqrt(4 * W)).to(dev)
    pk = lambda w: ops.split_hi16(ops.split_pack(w)) if mode == 2 else ops.split_pack(w)
    bfc, bpj = pk(wfc), pk(wpj)
    bias_fc = torch.randn(4 * W, generator=g).to(dev)
    bias_pj = torch.randn(W, generator=g).to(dev)
    res = torch.randn(M, W, generator=g).to(dev)
    # c_fc (training form: QuickGELU(h) and the saved derivative) -> c_proj
    for e in (N.EPI_BIAS_QGELU | N.QGELU_DERIV, N.EPI_BIAS_QGELU):
        y, d = ops.gemm(x, bfc, e, bias=bias_fc, want_out2=True)
        ys, ds = ops.gemm(x, bfc, e | N.OUT_SPLIT, bias=bias_fc, want_out2=True)
        assert torch.equal(ys.view(torch.int32), split_form(y).view(torch.int32)), f"c_fc split output, epi {e:#x}"
        assert torch.equal(ds, d)
    o = ops.gemm(y, bpj, N.EPI_BIAS_RES, bias=bias_pj, res=res)
    os_ = ops.gemm(ys, bpj, N.EPI_BIAS_RES | N.A_SPLIT, bias=bias_pj, res=res)
    assert torch.equal(os_, o), "c_proj on the pre-split A"
    st1, st2 = torch.empty(M, W // 64, 2, device=dev), torch.empty(M, W // 64, 2, device=dev)
    o1 = ops.gemm_ln(y, bpj, N.EPI_BIAS_RES, bias_pj, stats=st1, res=res)
    o2 = ops.gemm_ln(ys, bpj, N.EPI_BIAS_RES | N.A_SPLIT, bias_pj, stats=st2, res=res)
    assert torch.equal(o1, o2) and torch.equal(st1, st2)
    # dgelu (acc x the saved derivative) -> fc_dx
    aux = torch.rand(M, 4 * W, generator=g).to(dev)
    wfcT = pk(wfc.t().contiguous())
    wpjT = pk(wpj.t().contiguous())
    dh = ops.gemm(res, wpjT, N.EPI_DQGELU | N.QGELU_DERIV, aux=aux)
    dhs = ops.gemm(res, wpjT, N.EPI_DQGELU | N.QGELU_DERIV | N.OUT_SPLIT, aux=aux)
    assert torch.equal(dhs.view(torch.int32), split_form(dh).view(torch.int32)), "dgelu split output"
    assert torch.equal(ops.gemm(dhs, wfcT, N.EPI_NONE | N.A_SPLIT), ops.gemm(dh, wfcT, N.EPI_NONE)), "fc_dx"
    # the LayerNorm folds of c_fc with a split output
    gamma = (1.0 + 0.2 * torch.randn(W, generator=g)).to(dev)
    beta = (0.1 * torch.randn(W, generator=g)).to(dev)
    _, _, rnb = ops.ln_stats_merge(_partials(x), W)
    if mode == 2:
        wh, s, c = M_.ln_fold_weights(wfc.cpu(), bias_fc.cpu(), gamma.cpu(), beta.cpu(), torch.float32, dev,
                                      split=True, gamma_on_a=True)
        f, fd = ops.gemm_ln_gamma(x, wh, N.EPI_BIAS_QGELU | N.QGELU_DERIV, c, s, rnb, gamma, want_out2=True)
        fs, fds = ops.gemm_ln_gamma(x, wh, N.EPI_BIAS_QGELU | N.QGELU_DERIV | N.OUT_SPLIT, c, s, rnb, gamma,
                                    want_out2=True)
        assert torch.equal(fs.view(torch.int32), split_form(f).view(torch.int32)) and torch.equal(fds, fd)
        # the fold reading A pre-split as split(x * gamma): clipk_gemm_ln_stats_split's out2
        xs = split_form(x * gamma)
        fa, fda = ops.gemm_ln_gamma(xs, wh, N.EPI_BIAS_QGELU | N.QGELU_DERIV | N.A_SPLIT | N.OUT_SPLIT, c, s, rnb,
                                    gamma, want_out2=True)
        assert torch.equal(fa.view(torch.int32), fs.view(torch.int32)) and torch.equal(fda, fd), \
            "fold on the pre-split x * gamma"
        q, _ = ops.gemm_ln_gamma(x, wh, N.EPI_BIAS, c, s, rnb, gamma), None
        qa = ops.gemm_ln_gamma(xs, wh, N.EPI_BIAS | N.A_SPLIT, c, s, rnb, gamma)
        assert torch.equal(qa, q)
        st3 = torch.empty(M, W // 64, 2, device=dev)
        o3, o3s = ops.gemm_ln_stats_split(ys, bpj, N.EPI_BIAS_RES | N.A_SPLIT, bias_pj, st3, res, gamma)
        assert torch.equal(o3, o1) and torch.equal(st3, st1)
        assert torch.equal(o3s.view(torch.int32), split_form(o1 * gamma).view(torch.int32)), "stats_split out2"
    else:
        wp, s, c = M_.ln_fold_weights(wfc.cpu(), bias_fc.cpu(), gamma.cpu(), beta.cpu(), torch.float32, dev,
                                      split=True)
        f, fd = ops.gemm_ln(x, wp, N.EPI_BIAS_QGELU | N.QGELU_DERIV, c, colsum=s, rnb=rnb, want_out2=True)
        fs, fds = ops.gemm_ln(x, wp, N.EPI_BIAS_QGELU | N.QGELU_DERIV | N.OUT_SPLIT, c, colsum=s, rnb=rnb,
                              want_out2=True)
        assert torch.equal(fs.view(torch.int32), split_form(f).view(torch.int32)) and torch.equal(fds, fd)


def _partials(x):
    M, W = x.shape
    v = x.view(M, W // 64, 64).double()
    s = v.sum(2)
    mu = s / 64
    return torch.stack([s, ((v - mu[..., None]) ** 2).sum(2)], 2).float()


def test_presplit_flags_refused_where_not_built(dev):
    """Pre-split flags on a 16-bit / fp32 GEMM, on a 16-bit out, or with an epilogue no encoder
    hands off are refused before any launch (CLIPK_EINVAL / EDTYPE), never run as a plain GEMM."""
    lib = N.load()
    a = torch.randn(256, 512, device=dev)
    b16 = torch.randn(512, 512, device=dev).half()
    out = torch.empty(256, 512, device=dev)
    args = lambda ind, epi, b: (ind, N.F32, epi, 256, 512, 512, ops._p(a), 512, ops._p(b), 512, None, None, 512,
                                ops._p(out), 512, None, None, 0, 512, ops._stream())
    assert lib.clipk_gemm(*args(N.F16, N.EPI_NONE | N.A_SPLIT, b16)) < 0
    assert lib.clipk_gemm(*args(N.F32, N.EPI_NONE | N.OUT_SPLIT, a[:, :512].contiguous())) < 0
    assert lib.clipk_gemm(*args(N.F32S16, N.EPI_NONE | N.OUT_SPLIT, b16)) < 0  # EPI_NONE does not hand off split
    assert lib.clipk_gemm(*args(N.F32S16, N.EPI_NONE | 0x1000, b16)) < 0


@pytest.mark.parametrize("rows,W", [(47160, 512), (300, 512), (257, 768)])
def test_layernorm_bwd_split_copy(dev, rows, W):
    """The LayerNorm backward's pre-split copy of its fp32 output (lp dtype CLIPK_F32S: the A of
    proj_dx / out_dx under PREC fp32s) is bitwise split_form(dx), and dx itself is unchanged; at
    W 768 the 4-element lanes store half groups."""
    g = torch.Generator(device="cpu").manual_seed(rows + W)
    x = (torch.randn(rows, W, generator=g) + torch.randn(rows, 1, generator=g)).to(dev)
    dy = torch.randn(rows, W, generator=g).to(dev)
    dres = torch.randn(rows, W, generator=g).to(dev)
    w = (1 + 0.1 * torch.randn(W, generator=g)).to(dev)
    mean = x.mean(1)
    rstd = torch.rsqrt(x.var(1, unbiased=False) + 1e-5)
    dx0 = ops.layernorm_bwd(dy, x, w, mean, rstd, dres=dres)
    dx, lp = ops.layernorm_bwd(dy, x, w, mean, rstd, dres=dres, lp_dtype="split")
    assert torch.equal(dx, dx0)
    assert torch.equal(lp.view(torch.int32), split_form(dx).view(torch.int32))


@pytest.mark.parametrize("G,C,P,H,max_q", [(2, 37, 5, 8, 6), (1, 19, 16, 2, 7), (24, 300, 5, 8, 7)])
def test_attention_prefix_bwd_split_copy(dev, G, C, P, H, max_q):
    """The fp32 shared-prefix attention backward with grad dtype CLIPK_F32S (PREC fp32s: dq|dk|dv
    handed to the qkv input-grad GEMM pre-split) stores bitwise split_form of the fp32 backward's
    dq|dk|dv -- the rows the attention kernel writes and the prefix rows' reduced dK / dV -- and
    that GEMM on it (CLIPK_A_SPLIT) equals the GEMM on the fp32 values."""
    from test_kernels_gpu import prefix_case
    R, tiles, row_first, off, qlen, g = prefix_case(G, C, P, H, max_q, seed=G * 100 + C + P)
    W = H * 64
    qkv = torch.randn(G * R, 3 * W, generator=g).to(dev)
    tiles, row_first = tiles.to(dev), row_first.to(dev)
    o, lse = ops.attention_prefix(qkv, G, P, R, tiles, row_first, H, lse=True)
    dout = torch.randn(G * R, W, generator=g).to(dev)
    d32 = ops.attention_prefix_bwd(qkv, o, dout, lse, G, P, R, tiles, row_first, H, torch.float32)
    ds = ops.attention_prefix_bwd(qkv, o, dout, lse, G, P, R, tiles, row_first, H, torch.float32, split=True)
    assert torch.equal(ds.view(torch.int32), split_form(d32).view(torch.int32))
    w = _w16((W, 3 * W), g, 1 / math.sqrt(3 * W)).to(dev)
    wh = ops.split_hi16(ops.split_pack(w))
    assert torch.equal(ops.gemm(ds, wh, N.EPI_NONE | N.A_SPLIT), ops.gemm(d32, wh, N.EPI_NONE))


_T96_PROBE = r"""
import os, sys, math, torch
sys.path.insert(0, os.environ["FSP_ROOT"])
from fsp_amd import ops, _native as N
dev = torch.device("cuda", 0)
out = {}
for M in (4600, 5895):
    g = torch.Generator(device="cpu").manual_seed(M)
    a = torch.randn(M, 2048, generator=g).to(dev)
    b = (torch.randn(512, 2048, generator=g) / math.sqrt(2048)).half().float().to(dev)
    bias = torch.randn(512, generator=g).to(dev)
    res = torch.randn(M, 512, generator=g).to(dev)
    bh = ops.split_hi16(ops.split_pack(b))
    st = torch.empty(M, 8, 2, device=dev)
    out[M] = [ops.gemm(a, bh, N.EPI_NONE).cpu(), ops.gemm(a, bh, N.EPI_BIAS_RES, bias=bias, res=res).cpu(),
              ops.gemm_ln(a, bh, N.EPI_BIAS_RES, bias, stats=st, res=res).cpu(), st.cpu()]
torch.save(out, sys.argv[1])
"""


def test_gemm_t96_bitwise_t128(tmp_path):
    """The 96-row deep-ring tiles (batch-1 text N = 512 GEMMs: 188 -> 248 blocks) give the
    128x128 tiles' outputs bit for bit (the same per-element K order): the same GEMMs in two
    child processes, CLIPK_GEMM_T96 on and off (the knob is read once per process)."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    res = {}
    for t96 in ("1", "0"):
        f = str(tmp_path / f"t96_{t96}.pt")
        env = dict(os.environ, FSP_ROOT=root, CLIPK_GEMM_T96=t96)
        p = subprocess.run([sys.executable, "-c", _T96_PROBE, f], env=env, capture_output=True, text=True, timeout=240)
        assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-2000:]
        res[t96] = torch.load(f, weights_only=True)
    for M in (4600, 5895):
        for i, (x, y) in enumerate(zip(res["1"][M], res["0"][M])):
            assert torch.equal(x, y), f"M {M} output {i}: {int((x != y).sum())} differ"
