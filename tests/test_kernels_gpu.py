"""Per-kernel numerics on the GPU: each HIP kernel vs a plain PyTorch fp32 reference of
the same op (float kernels), through the C-ABI. Tolerances are stated per dtype:
fp32 kernels (f32-input MFMA / fp32 VALU) 2e-5 relative-to-scale, fp16 1e-2, bf16 3e-2
(all relative to the reference's max |value|)."""
import math
import os
import subprocess
import sys

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from fsp_amd import ops, _native as N

pytestmark = pytest.mark.gpu

TOL = {torch.float32: 2e-5, torch.float16: 1e-2, torch.bfloat16: 3e-2}


def close(out, ref, dtype, what):
    out = out.float()
    ref = ref.float()
    scale = ref.abs().max().item() + 1e-12
    err = (out - ref).abs().max().item() / scale
    assert err <= TOL[dtype], f"{what}: rel err {err:.3e} > {TOL[dtype]} ({dtype})"


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16, torch.float32])
@pytest.mark.parametrize("M,Nn,K", [(300, 384, 192), (128, 128, 64), (1, 256, 512), (517, 1536, 512)])
def test_gemm_epilogues(dev, dtype, M, Nn, K):
    g = torch.Generator(device="cpu").manual_seed(M * 7 + Nn + K)
    a = torch.randn(M, K, generator=g).to(dev)
    b = (torch.randn(Nn, K, generator=g) / math.sqrt(K)).to(dev)
    bias = torch.randn(Nn, generator=g).to(dev)
    res = torch.randn(M, Nn, generator=g).to(dev)
    A, Bm = a.to(dtype), b.to(dtype)
    ref = A.float() @ Bm.float().t()
    close(ops.gemm(A, Bm, N.EPI_NONE, torch.float32), ref, dtype, "none")
    close(ops.gemm(A, Bm, N.EPI_BIAS, dtype, bias=bias), ref + bias, dtype, "bias")
    close(ops.gemm(A, Bm, N.EPI_BIAS_RES, torch.float32, bias=bias, res=res), ref + bias + res, dtype, "res")
    g_out, h_out = ops.gemm(A, Bm, N.EPI_BIAS_QGELU, dtype, bias=bias, want_out2=True)
    hr = ref + bias
    close(h_out, hr, dtype, "qgelu.h")
    close(g_out, hr * torch.sigmoid(1.702 * hr), dtype, "qgelu.g")
    aux = torch.randn(M, Nn, generator=g).to(dev).to(dtype)
    s = torch.sigmoid(1.702 * aux.float())
    dref = ref * (s + 1.702 * aux.float() * s * (1 - s))
    close(ops.gemm(A, Bm, N.EPI_DQGELU, dtype, aux=aux), dref, dtype, "dqgelu")


def test_gemm_identity_asymmetric(dev):
    """A = I with an asymmetric B catches a transposed C write (guide §3)."""
    K = 128
    A = torch.eye(K, device=dev, dtype=torch.float16)
    B = (torch.arange(256 * K, device=dev, dtype=torch.float32).reshape(256, K) % 97).to(torch.float16)
    out = ops.gemm(A, B, N.EPI_NONE, torch.float32)
    assert torch.equal(out, B.float().t()[:K])


def test_gemm_rejects_bad_shapes(dev):
    A = torch.randn(10, 64, device=dev, dtype=torch.float16)
    B = torch.randn(100, 64, device=dev, dtype=torch.float16)  # N % 128 != 0
    with pytest.raises(N.ClipkError):
        ops.gemm(A, B)


@pytest.mark.parametrize("W", [128, 512, 768, 1024])
@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16, torch.float32])
def test_layernorm_fwd_bwd(dev, W, dtype):
    g = torch.Generator().manual_seed(W)
    x = (torch.randn(37, W, generator=g) * 3 + 1).to(dev)
    w = (1 + 0.1 * torch.randn(W, generator=g)).to(dev)
    b = (0.1 * torch.randn(W, generator=g)).to(dev)
    out, mean, rstd = ops.layernorm(x, w, b, dtype, stats=True)
    xr = x.clone().requires_grad_(True)
    ref = F.layer_norm(xr, (W,), w, b, 1e-5)
    close(out, ref, dtype, "ln fwd")
    dy = torch.randn(37, W, generator=g).to(dev)
    dres = torch.randn(37, W, generator=g).to(dev)
    ref.backward(dy)
    dx = ops.layernorm_bwd(dy, x, w, mean, rstd, dres=dres)
    close(dx, xr.grad + dres, torch.float32, "ln bwd")
    rows = torch.tensor([3, 0, 36], device=dev, dtype=torch.int32)
    og = ops.layernorm(x, w, b, torch.float32, rows=rows)
    close(og, F.layer_norm(x[rows.long()], (W,), w, b, 1e-5), torch.float32, "ln gather")


@pytest.mark.parametrize("xdt", [torch.float16, torch.bfloat16])
def test_layernorm_16bit_residual(dev, xdt):
    """16-bit residual stream (PREC fp16/bf16 text encoder): LN fwd/bwd read x in the
    activation dtype, statistics in fp32; vs torch fp32 on the same rounded x."""
    W = 512
    g = torch.Generator().manual_seed(11)
    x = (torch.randn(41, W, generator=g) * 3 + 1).to(dev).to(xdt)
    w = (1 + 0.1 * torch.randn(W, generator=g)).to(dev)
    b = (0.1 * torch.randn(W, generator=g)).to(dev)
    out, mean, rstd = ops.layernorm(x, w, b, xdt, stats=True)
    xr = x.float().clone().requires_grad_(True)
    ref = F.layer_norm(xr, (W,), w, b, 1e-5)
    close(out, ref, xdt, "ln16 fwd")
    dy = torch.randn(41, W, generator=g).to(dev).to(torch.bfloat16)
    ref.backward(dy.float())
    dx = ops.layernorm_bwd(dy, x, w, mean, rstd)
    close(dx, xr.grad, torch.float32, "ln16 bwd")  # same rounded inputs, fp32 math


def test_layernorm_bwd_16bit_residual_grad(dev):
    """16-bit residual-gradient stream (CLIPK_TEXT_DRES16): dres (bf16) updated in place with
    LN'(dy), and the optional fp32 copy; vs torch fp32 on the same rounded inputs."""
    W = 512
    g = torch.Generator().manual_seed(12)
    x = (torch.randn(45, W, generator=g) * 2).to(dev).to(torch.float16)
    w = (1 + 0.1 * torch.randn(W, generator=g)).to(dev)
    b = torch.zeros(W, device=dev)
    _, mean, rstd = ops.layernorm(x, w, b, torch.float16, stats=True)
    xr = x.float().clone().requires_grad_(True)
    ref = F.layer_norm(xr, (W,), w, b, 1e-5)
    dy = torch.randn(45, W, generator=g).to(dev).to(torch.bfloat16)
    ref.backward(dy.float())
    dres = torch.randn(45, W, generator=g).to(dev).to(torch.bfloat16)
    want = xr.grad + dres.float()
    dx = torch.empty(45, W, device=dev)
    got = ops.layernorm_bwd_lp_(dy, x, w, mean, rstd, dres, dx=dx)
    assert got.data_ptr() == dres.data_ptr()
    close(got, want, torch.bfloat16, "ln bwd dres16")
    close(dx, want, torch.float16, "ln bwd dres16 fp32 copy")


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("M,Nn,K", [(40000, 512, 2048), (300, 256, 512), (8192, 2048, 512), (1, 128, 64)])
def test_gemm_a_qgelu(dev, dtype, M, Nn, K):
    """CLIPK_A_QGELU: out = quickgelu(A) . B^T + bias + res, QuickGELU applied to the 16-bit A
    chunks while they are staged (the text c_proj forward reading c_fc's pre-activation);
    vs torch on the same 16-bit rounding of quickgelu(A)."""
    g = torch.Generator().manual_seed(M + K)
    h = (torch.randn(M, K, generator=g) * 2).to(dev).to(dtype)
    B = (torch.randn(Nn, K, generator=g) / math.sqrt(K)).to(dev).to(dtype)
    bias = torch.randn(Nn, generator=g).to(dev)
    res = torch.randn(M, Nn, generator=g).to(dev).to(dtype)
    hf = h.float()
    a = (hf * torch.sigmoid(1.702 * hf)).to(dtype).float()
    ref = a @ B.float().t() + bias + res.float()
    close(ops.gemm(h, B, N.EPI_BIAS_RES | N.A_QGELU, dtype, bias=bias, res=res), ref, dtype, f"a_qgelu M{M}")
    resf = res.float()
    close(ops.gemm(h, B, N.EPI_BIAS_RES | N.A_QGELU, torch.float32, bias=bias, res=resf),
          a @ B.float().t() + bias + resf, dtype, f"a_qgelu f32 M{M}")
    with pytest.raises(N.ClipkError):
        ops.gemm(h, B, N.EPI_NONE | N.A_QGELU, torch.float32)


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
def test_gemm_bias_res_16bit(dev, dtype):
    """BIAS_RES with a 16-bit residual stream: out (dtype) = A.B^T + bias + res (dtype)."""
    for M in (300, 40000):
        g = torch.Generator().manual_seed(M)
        A = torch.randn(M, 512, generator=g).to(dev).to(dtype)
        B = (torch.randn(512, 512, generator=g) / math.sqrt(512)).to(dev).to(dtype)
        bias = torch.randn(512, generator=g).to(dev)
        res = torch.randn(M, 512, generator=g).to(dev).to(dtype)
        ref = A.float() @ B.float().t() + bias + res.float()
        close(ops.gemm(A, B, N.EPI_BIAS_RES, dtype, bias=bias, res=res), ref, dtype, f"res16 M{M}")


@pytest.mark.parametrize("K", [512, 2048])
def test_gemm_bench_shape_n512(dev, K):
    """N = 512 at the headline's 47,160 rows (192x256 ping-pong tiles, 1.92 rounds of CUs): the
    input-grad form (fp16 out) and the 16-bit residual form, every row against torch fp32."""
    M, dtype = 47160, torch.float16
    g = torch.Generator().manual_seed(K)
    A = torch.randn(M, K, generator=g).to(dev).to(dtype)
    B = (torch.randn(512, K, generator=g) / math.sqrt(K)).to(dev).to(dtype)
    bias = torch.randn(512, generator=g).to(dev)
    res = torch.randn(M, 512, generator=g).to(dev).to(dtype)
    ref = A.float() @ B.float().t()
    close(ops.gemm(A, B, N.EPI_NONE, dtype), ref, dtype, f"n512 none K{K}")
    close(ops.gemm(A, B, N.EPI_BIAS_RES, dtype, bias=bias, res=res), ref + bias + res.float(), dtype,
          f"n512 res16 K{K}")


def attn_ref(qkv, nseq, L, H, causal):
    W = H * 64
    q, k, v = qkv.float().view(nseq, L, 3, H, 64).permute(2, 0, 3, 1, 4)
    s = q @ k.transpose(-1, -2) / 8.0
    if causal:
        s = s + torch.full((L, L), float("-inf"), device=qkv.device).triu(1)
    lse = torch.logsumexp(s, -1)
    o = torch.softmax(s, -1) @ v
    return o.permute(0, 2, 1, 3).reshape(nseq * L, W), lse.permute(0, 2, 1).reshape(nseq * L, H)


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16, torch.float32])
@pytest.mark.parametrize("nseq,L,H,causal", [(7, 11, 8, 1), (5, 23, 2, 1), (3, 50, 4, 1), (2, 77, 8, 1),
                                             (2, 197, 12, 0), (1, 257, 2, 0), (3, 5, 2, 0), (2, 577, 4, 0),
                                             (2, 130, 2, 1)])
def test_attention_fwd(dev, dtype, nseq, L, H, causal):
    g = torch.Generator().manual_seed(L * H)
    qkv = torch.randn(nseq * L, 3 * H * 64, generator=g).to(dev).to(dtype)
    o, lse = ops.attention(qkv, nseq, L, H, causal, lse=True)
    ro, rl = attn_ref(qkv, nseq, L, H, causal)
    close(o, ro, dtype, "attn out")
    close(lse, rl, torch.float16 if dtype != torch.float32 else dtype, "attn lse")


@pytest.mark.parametrize("dtype,gdtype", [(torch.float16, torch.bfloat16), (torch.float16, torch.float16),
                                         (torch.bfloat16, torch.bfloat16), (torch.float32, torch.float32)])
@pytest.mark.parametrize("nseq,L,H,causal", [(6, 11, 8, 1), (3, 23, 2, 1), (2, 64, 2, 1), (4, 5, 2, 1),
                                             (2, 77, 8, 1), (3, 50, 4, 0), (2, 100, 2, 1), (2, 201, 12, 0),
                                             (1, 257, 2, 0), (2, 33, 2, 0)])
def test_attention_bwd(dev, dtype, gdtype, nseq, L, H, causal):
    """L <= 16: one MFMA tile; longer (text L_eff 17..77, the prompted ViT's 50..600 rows):
    the two-pass kernels (MFMA for 16-bit, VALU for fp32)."""
    g = torch.Generator().manual_seed(L + 100 * H)
    qkv = torch.randn(nseq * L, 3 * H * 64, generator=g).to(dev).to(dtype)
    o, lse = ops.attention(qkv, nseq, L, H, causal, lse=True)
    do = torch.randn(nseq * L, H * 64, generator=g).to(dev).to(gdtype)
    dqkv = ops.attention_bwd(qkv, o, do, lse, nseq, L, H, causal, gdtype)
    qr = qkv.float().clone().requires_grad_(True)
    ro, _ = attn_ref(qr, nseq, L, H, causal)
    ro.backward(do.float())
    close(dqkv, qr.grad, gdtype if dtype != torch.float32 else dtype, "attn bwd")


@pytest.mark.parametrize("dtype", [torch.float32, torch.float16, torch.bfloat16])
def test_rows_inject_collect(dev, dtype):
    """Deep-prompt row replacement and its gradient (sum over the sequences sharing a prompt
    row, replaced rows zeroed)."""
    g = torch.Generator().manual_seed(5)
    n_ctx, n_per, W, rows_total = 3, 5, 256, 40
    rows = torch.randperm(rows_total, generator=g)[: n_ctx * n_per].to(torch.int32)
    src = torch.randn(n_ctx, W, generator=g)
    dst = torch.randn(rows_total, W, generator=g).to(dtype)
    ref = dst.clone()
    for p in range(n_ctx):
        for i in range(n_per):
            ref[rows[p * n_per + i]] = src[p].to(dtype)
    out = ops.rows_inject(src.to(dev), rows.to(dev), dst.to(dev), n_per)
    assert torch.equal(out.cpu(), ref)
    grad = torch.randn(rows_total, W, generator=g).to(dtype)
    want = torch.stack([sum(grad[rows[p * n_per + i]].float() for i in range(n_per)) for p in range(n_ctx)])
    gd = grad.to(dev)
    twin = grad.float().to(dev)
    got = ops.rows_collect(gd, rows.to(dev), n_ctx, n_per, src2=twin)
    torch.testing.assert_close(got.cpu(), want, rtol=1e-6, atol=1e-5)
    zeroed = grad.clone()
    zeroed[rows.long()] = 0
    assert torch.equal(gd.cpu(), zeroed) and torch.equal(twin.cpu(), zeroed.float())


@pytest.mark.parametrize("patch,res", [(16, 32), (32, 64), (14, 28)])
def test_im2col_patch_gemm(dev, patch, res):
    g = torch.Generator().manual_seed(patch)
    img = torch.randn(2, 3, res, res, generator=g).to(dev)
    D = 128
    w = (torch.randn(D, 3, patch, patch, generator=g) * 0.05).to(dev)
    k = 3 * patch * patch
    Kp = (k + 63) // 64 * 64
    wp = torch.zeros(D, Kp, device=dev)
    wp[:, :k] = w.reshape(D, k)
    cols = ops.im2col(img, patch, Kp, torch.float32)
    out = ops.gemm(cols, wp, N.EPI_NONE, torch.float32)
    ref = F.conv2d(img, w, stride=patch).flatten(2).transpose(1, 2).reshape(-1, D)
    close(out, ref, torch.float32, "patch embed")


def test_cosine_logits_ce_focal(dev):
    g = torch.Generator().manual_seed(0)
    B, C, E = 5, 37, 512
    imf = torch.randn(B, E, generator=g).to(dev)
    for per_image in (0, 1):
        txt = torch.randn(B * C if per_image else C, E, generator=g).to(dev).requires_grad_(True)
        scale = 100.0
        logits, inv_t, inv_i = ops.cosine_logits(imf, txt.detach(), scale, per_image, C)
        tn = txt / txt.norm(dim=-1, keepdim=True)
        ifn = imf / imf.norm(dim=-1, keepdim=True)
        ref = scale * (torch.einsum("be,bce->bc", ifn, tn.view(B, C, E)) if per_image else ifn @ tn.t())
        close(logits, ref, torch.float32, "logits")
        y = torch.from_numpy(__import__("numpy").random.RandomState(1).randint(0, C, B)).to(dev)
        alpha = torch.rand(C, generator=g).to(dev) + 0.5
        for focal in (0, 1):
            lr = ref.detach().clone().requires_grad_(True)
            if focal:
                ce = F.cross_entropy(lr, y, reduction="none")
                loss = (alpha[y] * (1 - torch.exp(-ce)) ** 2 * ce).mean()
            else:
                loss = F.cross_entropy(lr, y)
            loss.backward()
            row, dl = ops.ce_loss(logits, y, alpha if focal else None, 2.0, bool(focal))
            assert abs(row.mean().item() - loss.item()) < 1e-4 * max(1.0, abs(loss.item()))
            close(dl, lr.grad, torch.float32, "dlogits")
        txt.grad = None
        dlg = torch.randn(B, C, generator=g).to(dev)
        ref.backward(dlg)
        dtxt = ops.cosine_logits_bwd(imf, txt.detach(), inv_t, inv_i, dlg, scale, per_image)
        close(dtxt, txt.grad, torch.float32, "dtxt")


@pytest.mark.parametrize("B,V,Wd", [(4, 512, 512), (1, 768, 768), (3, 1024, 640), (2, 96, 80)])
def test_meta_net_and_sgd(dev, B, V, Wd):
    g = torch.Generator().manual_seed(3)
    Hd = V // 16
    x = torch.randn(B, V, generator=g).to(dev)
    w1 = (torch.randn(Hd, V, generator=g) * 0.05).to(dev).requires_grad_(True)
    b1 = (torch.randn(Hd, generator=g) * 0.05).to(dev).requires_grad_(True)
    w2 = (torch.randn(Wd, Hd, generator=g) * 0.1).to(dev).requires_grad_(True)
    b2 = (torch.randn(Wd, generator=g) * 0.05).to(dev).requires_grad_(True)
    h, y = ops.meta_net(x, w1.detach(), b1.detach(), w2.detach(), b2.detach())
    ref = torch.relu(x @ w1.t() + b1) @ w2.t() + b2
    close(y, ref, torch.float32, "meta fwd")
    dy = torch.randn(B, Wd, generator=g).to(dev)
    ref.backward(dy)
    dw1, db1, dw2, db2 = ops.meta_net_bwd(x, h, w2.detach(), dy, V, Hd, Wd)
    for a, r, n in ((dw1, w1.grad, "dw1"), (db1, b1.grad, "db1"), (dw2, w2.grad, "dw2"), (db2, b2.grad, "db2")):
        close(a, r, torch.float32, n)
    p = torch.randn(1000, generator=g).to(dev)
    gr = torch.randn(1000, generator=g).to(dev)
    buf = torch.zeros_like(p)
    pr = p.clone().requires_grad_(True)
    opt = torch.optim.SGD([pr], lr=0.002, momentum=0.9, weight_decay=5e-4)
    for step in range(3):
        pr.grad = gr.clone()
        opt.step()
        ops.sgd_step(p, gr, buf, 0.002, 0.9, 5e-4, step > 0)
    close(p, pr.detach(), torch.float32, "sgd")
    # the multi-tensor launch (FusedSGD's path): bitwise the per-tensor update, ragged sizes
    sizes = [1000, 17, 4096, 1, 2048]
    ps = [torch.randn(n, generator=g).to(dev) for n in sizes]
    gs = [torch.randn(n, generator=g).to(dev) for n in sizes]
    pa, ba = [t.clone() for t in ps], [torch.zeros_like(t) for t in ps]
    pb, bb = [t.clone() for t in ps], [torch.zeros_like(t) for t in ps]
    for step in range(3):
        for t, gt, mt in zip(pa, gs, ba):
            ops.sgd_step(t, gt, mt, 0.002, 0.9, 5e-4, step > 0)
        ops.sgd_step_multi(pb, gs, bb, 0.002, 0.9, 5e-4, [step > 0] * len(sizes))
    for t1, t2, m1, m2 in zip(pa, pb, ba, bb):
        assert torch.equal(t1, t2) and torch.equal(m1, m2)
    # the gradient scale of a SUM all-reduce folded into the update (clipk_sgd_step_multi_scaled):
    # bitwise the update on the pre-scaled gradients for a power-of-two scale
    pc, bc = [t.clone() for t in ps], [torch.zeros_like(t) for t in ps]
    pd, bd = [t.clone() for t in ps], [torch.zeros_like(t) for t in ps]
    for step in range(3):
        ops.sgd_step_multi(pc, [gt * 0.125 for gt in gs], bc, 0.002, 0.9, 5e-4, [step > 0] * len(sizes))
        ops.sgd_step_multi(pd, gs, bd, 0.002, 0.9, 5e-4, [step > 0] * len(sizes), grad_scale=0.125)
    for t1, t2, m1, m2 in zip(pc, pd, bc, bd):
        assert torch.equal(t1, t2) and torch.equal(m1, m2)


@pytest.mark.parametrize("B,V,Wd", [(4, 512, 512), (8, 512, 512), (1, 768, 768), (2, 96, 80)])
def test_meta_net_fwd_norm(dev, B, V, Wd):
    """clipk_meta_net_fwd_norm: xn = x / |x| (cocoop.py:238) and the Meta-Net on it in one launch,
    against torch's imf / imf.norm() and the un-normalised entry point on that."""
    g = torch.Generator().manual_seed(5)
    Hd = V // 16
    x = (torch.randn(B, V, generator=g) * 3).to(dev)
    w1 = (torch.randn(Hd, V, generator=g) * 0.05).to(dev)
    b1 = (torch.randn(Hd, generator=g) * 0.05).to(dev)
    w2 = (torch.randn(Wd, Hd, generator=g) * 0.1).to(dev)
    b2 = (torch.randn(Wd, generator=g) * 0.05).to(dev)
    xn, h, y = ops.meta_net(x, w1, b1, w2, b2, normalize=True)
    ref = x / x.norm(dim=-1, keepdim=True)
    torch.testing.assert_close(xn, ref, rtol=2e-6, atol=1e-7)
    h2, y2 = ops.meta_net(ref, w1, b1, w2, b2)
    torch.testing.assert_close(y, y2, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(h, h2, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("B,C", [(8, 1000), (1, 1000), (13, 37)])
@pytest.mark.parametrize("reduction", ["mean", "sum"])
def test_ce_loss_reduce(dev, B, C, reduction):
    """clipk_ce_loss_reduce: the batch reduction in the loss launch -- dlogits bitwise the
    per-row kernel's, the loss = the row-order sum (/ B) of its row losses."""
    g = torch.Generator().manual_seed(B + C)
    logits = (torch.randn(B, C, generator=g) * 4).to(dev)
    y = torch.randint(0, C, (B,), generator=g).to(dev)
    alpha = (torch.rand(C, generator=g) + 0.5).to(dev)
    for focal in (False, True):
        a = alpha if focal else None
        scale = 1.0 / B if reduction == "mean" else 1.0
        row, dl = ops.ce_loss(logits, y, a, 2.0, focal, grad_scale=scale)
        loss, dl2 = ops.ce_loss_reduce(logits, y, a, 2.0, focal, reduction=reduction)
        assert torch.equal(dl, dl2)
        s = row[0].clone()
        for b in range(1, B):
            s = s + row[b]
        ref = s * (1.0 / B) if reduction == "mean" else s
        assert torch.equal(loss, ref), (loss.item(), ref.item())


def test_status_take(dev):
    """clipk_status_take: the flags reach the pinned host word and are cleared, stream-ordered."""
    flags = torch.tensor([6], dtype=torch.int32, device=dev)
    host = torch.zeros(1, dtype=torch.int32, pin_memory=True)
    ops.status_take(flags, host)
    torch.cuda.synchronize()
    assert int(host[0]) == 6 and int(flags.item()) == 0
    ops.status_take(flags, host)
    torch.cuda.synchronize()
    assert int(host[0]) == 0


@pytest.mark.parametrize("cfg", [0, 1, 2, 3, 6])
@pytest.mark.parametrize("Nn,K", [(2048, 512), (512, 2048)])
def test_gemm_large_m_every_config(dev, cfg, Nn, K):
    """Bench-scale M (persistent / ring paths engage when tiles > 2x CUs) vs torch fp32."""
    lib = N.load()
    M = 40000
    g = torch.Generator(device="cpu").manual_seed(cfg * 31 + Nn)
    A = torch.randn(M, K, generator=g).to(dev).to(torch.float16)
    B = (torch.randn(Nn, K, generator=g) / math.sqrt(K)).to(dev).to(torch.float16)
    bias = torch.randn(Nn, generator=g).to(dev)
    res = torch.randn(M, Nn, generator=g).to(dev)
    aux = torch.randn(M, Nn, generator=g).to(dev).to(torch.float16)
    ref = A.float() @ B.float().t()
    try:
        N.check(lib.clipk_gemm_set_config(cfg), "set_config")
        close(ops.gemm(A, B, N.EPI_NONE, torch.float32), ref, torch.float16, f"cfg{cfg} none")
        close(ops.gemm(A, B, N.EPI_BIAS_RES, torch.float32, bias=bias, res=res), ref + bias + res,
              torch.float16, f"cfg{cfg} res")
        gq, hq = ops.gemm(A, B, N.EPI_BIAS_QGELU, torch.float16, bias=bias, want_out2=True)
        close(hq, ref + bias, torch.float16, f"cfg{cfg} qgelu.h")
        hr = ref + bias
        close(gq, hr * torch.sigmoid(1.702 * hr), torch.float16, f"cfg{cfg} qgelu.g")
        close(ops.gemm(A, B, N.EPI_BIAS, torch.bfloat16, bias=bias), ref + bias, torch.bfloat16, f"cfg{cfg} bias bf16")
        Ab, Bb = A.to(torch.bfloat16), B.to(torch.bfloat16)
        refb = Ab.float() @ Bb.float().t()
        s = torch.sigmoid(1.702 * aux.float())
        close(ops.gemm(Ab, Bb, N.EPI_DQGELU, torch.bfloat16, aux=aux),
              refb * (s + 1.702 * aux.float() * s * (1 - s)), torch.bfloat16, f"cfg{cfg} dqgelu")
    finally:
        lib.clipk_gemm_set_config(-1)


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("Nn,K", [(768, 3072), (768, 2304), (768, 768), (2304, 768), (3072, 768)])
def test_gemm_large_m_w768(dev, dtype, Nn, K):
    """The W = 768 text GEMMs of BASELINE configs 4 / 5 at their full-size M (C = 1,000 classes:
    ~44k packed rows), automatic tile choice (the persistent / ping-pong 192- and 256-row
    tiles), every epilogue the text encoder uses on that shape, 16-bit residual stream, vs a
    torch fp32 reference."""
    M = 44000
    g = torch.Generator(device="cpu").manual_seed(Nn * 3 + K)
    A = torch.randn(M, K, generator=g).to(dev).to(dtype)
    B = (torch.randn(Nn, K, generator=g) / math.sqrt(K)).to(dev).to(dtype)
    bias = torch.randn(Nn, generator=g).to(dev)
    res = torch.randn(M, Nn, generator=g).to(dev).to(dtype)
    aux = torch.randn(M, Nn, generator=g).to(dev).to(dtype)
    ref = A.float() @ B.float().t()
    close(ops.gemm(A, B, N.EPI_NONE, dtype), ref, dtype, f"{Nn}x{K} none")
    close(ops.gemm(A, B, N.EPI_NONE, torch.float32), ref, dtype, f"{Nn}x{K} none f32")
    close(ops.gemm(A, B, N.EPI_BIAS, dtype, bias=bias), ref + bias, dtype, f"{Nn}x{K} bias")
    close(ops.gemm(A, B, N.EPI_BIAS_RES, dtype, bias=bias, res=res), ref + bias + res.float(), dtype,
          f"{Nn}x{K} res16")
    gq, hq = ops.gemm(A, B, N.EPI_BIAS_QGELU, dtype, bias=bias, want_out2=True)
    hr = ref + bias
    close(hq, hr, dtype, f"{Nn}x{K} qgelu.h")
    close(gq, hr * torch.sigmoid(1.702 * hr), dtype, f"{Nn}x{K} qgelu.g")
    s = torch.sigmoid(1.702 * aux.float())
    close(ops.gemm(A, B, N.EPI_DQGELU, dtype, aux=aux), ref * (s + 1.702 * aux.float() * s * (1 - s)), dtype,
          f"{Nn}x{K} dqgelu")


@pytest.mark.parametrize("M,Nn,K", [(300, 384, 192), (517, 1536, 512), (4600, 768, 3072), (47160, 512, 2048),
                                     (47160, 2048, 512), (8000, 512, 512)])
def test_gemm_split_fp32_class(dev, M, Nn, K):
    """PREC fp32s GEMM (CLIPK_F32S: fp32 A split into fp16 hi + lo in registers, split-packed B,
    3 fp16 MFMAs per product) against an fp64 reference, every epilogue: within 4e-6 of the
    output scale (measured 3e-7 .. 1.8e-6, growing with K; the dropped lo x lo term is ~2^-22 of
    each product) -- the fp32 class, two orders of magnitude under fp16 operands; the 128x128
    grids, the 4-slot ring and the 192x256 ping-pong tiles all run here."""
    g = torch.Generator(device="cpu").manual_seed(M + Nn + K)
    a = torch.randn(M, K, generator=g).to(dev)
    b = (torch.randn(Nn, K, generator=g) * 0.03).to(dev)  # CLIP-like weight scale
    bias = torch.randn(Nn, generator=g).to(dev)
    res = torch.randn(M, Nn, generator=g).to(dev)
    aux = torch.randn(M, Nn, generator=g).to(dev)
    bp = ops.split_pack(b)
    ref = a.double() @ b.double().t()
    tol = 4e-6

    def chk(out, r, what):
        err = ((out.double() - r).abs().max() / (r.abs().max() + 1e-30)).item()
        assert err <= tol, f"{what}: rel err {err:.3e} > {tol}"
        return err
    e_none = chk(ops.gemm(a, bp, N.EPI_NONE), ref, "none")
    chk(ops.gemm(a, bp, N.EPI_BIAS, bias=bias), ref + bias.double(), "bias")
    chk(ops.gemm(a, bp, N.EPI_BIAS_RES, bias=bias, res=res), ref + bias.double() + res.double(), "res")
    gq, hq = ops.gemm(a, bp, N.EPI_BIAS_QGELU, bias=bias, want_out2=True)
    hr = ref + bias.double()
    chk(hq, hr, "qgelu.h")
    chk(gq, hr * torch.sigmoid(1.702 * hr), "qgelu.g")
    s = torch.sigmoid(1.702 * aux.double())
    chk(ops.gemm(a, bp, N.EPI_DQGELU, aux=aux), ref * (s + 1.702 * aux.double() * s * (1 - s)), "dqgelu")
    # for scale: the fp16 operands' error on the same product is ~1e-3
    e16 = ((ops.gemm(a.half(), b.half(), N.EPI_NONE).double() - ref).abs().max() / ref.abs().max()).item()
    e32 = ((ops.gemm(a, b, N.EPI_NONE).double() - ref).abs().max() / ref.abs().max()).item()
    print(f"split {M}x{Nn}x{K}: {e_none:.2e}  f32 MFMA: {e32:.2e}  fp16: {e16:.2e}")
    assert e_none * 50 < e16


@pytest.mark.parametrize("prec", [torch.float16, torch.bfloat16, torch.float32, "fp32s"])
@pytest.mark.parametrize("M", [300, 6000, 47160])
def test_gemm_qgelu_deriv_pair(dev, prec, M):
    """CLIPK_QGELU_DERIV (training's c_fc / dgelu pair): EPI_BIAS_QGELU writes out2 =
    quickgelu'(acc + bias) beside out = quickgelu(acc + bias), and EPI_DQGELU with the flag is
    out = acc * aux; vs torch fp32 of the same ops (tolerance per dtype; fp32s 4e-6), on the small-M,
    128x128 and ping-pong tiles. The QuickGELU output is bitwise the plain epilogue's."""
    Nn, K = 2048, 512
    g = torch.Generator(device="cpu").manual_seed(M)
    a = torch.randn(M, K, generator=g).to(dev)
    w = (torch.randn(Nn, K, generator=g) / math.sqrt(K)).to(dev)
    bias = (0.3 * torch.randn(Nn, generator=g)).to(dev)
    dy = torch.randn(M, K, generator=g).to(dev)  # dgelu: dY [M, W] . Wproj^T [W -> 4W]
    wproj = (torch.randn(Nn, K, generator=g) / math.sqrt(K)).to(dev)
    if prec == "fp32s":
        A, B, Dy, Wp, odt, tol = a, ops.split_pack(w), dy, ops.split_pack(wproj), torch.float32, 4e-6
        ref = a.double() @ w.double().t() + bias.double()
        acc = dy.double() @ wproj.double().t()
    else:
        A, B, Dy, Wp, odt, tol = a.to(prec), w.to(prec), dy.to(prec), wproj.to(prec), prec, TOL[prec]
        ref = A.double() @ B.double().t() + bias.double()
        acc = Dy.double() @ Wp.double().t()
    sg = torch.sigmoid(1.702 * ref)
    gq, dq = ops.gemm(A, B, N.EPI_BIAS_QGELU | N.QGELU_DERIV, odt, bias=bias, want_out2=True)
    g0 = ops.gemm(A, B, N.EPI_BIAS_QGELU, odt, bias=bias)
    assert torch.equal(gq, g0)
    scale = lambda r: r.abs().max().item() + 1e-12
    e_g = ((gq.double() - ref * sg).abs().max() / scale(ref * sg)).item()
    dref = sg * (1 + 1.702 * ref * (1 - sg))
    e_d = ((dq.double() - dref).abs().max() / scale(dref)).item()
    assert e_g <= tol and e_d <= tol, f"qgelu {e_g:.3e} deriv {e_d:.3e} > {tol}"
    out = ops.gemm(Dy, Wp, N.EPI_DQGELU | N.QGELU_DERIV, odt, aux=dq)
    want = acc * dq.double()
    e_o = ((out.double() - want).abs().max() / scale(want)).item()
    assert e_o <= tol, f"dmul {e_o:.3e} > {tol}"
    with pytest.raises(N.ClipkError):  # the flag means nothing to the other epilogues
        ops.gemm(A, B, N.EPI_BIAS | N.QGELU_DERIV, odt, bias=bias)


@pytest.mark.parametrize("M", [96, 1576, 47160])
def test_gemm_split_parts_exact(dev, M):
    """The in-register split itself, bit for bit: with B = I (packed hi = 64, lo = 0) every output
    is 64 (hi + lo) / 64 with hi = fp16(x), lo = fp16(x - hi) -- exact in fp32 -- so the result
    must equal the numpy split of A exactly, on the small-M, 128x128 and ping-pong tiles."""
    K = 512
    g = torch.Generator(device="cpu").manual_seed(M)
    a = torch.randn(M, K, generator=g) * torch.exp2(torch.randint(-6, 7, (M, K), generator=g).float())
    x = a.numpy()
    hi = x.astype(np.float16)
    lo = (x - hi.astype(np.float32)).astype(np.float16)
    want = hi.astype(np.float32) + lo.astype(np.float32)
    out = ops.gemm(a.to(dev), ops.split_pack(torch.eye(K).to(dev)), N.EPI_NONE).cpu().numpy()
    bad = int((out != want).sum())
    assert bad == 0, f"{bad} of {out.size} outputs differ from hi + lo"
    assert np.abs(want - x).max() <= np.abs(x).max() * 2.0 ** -21


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16])
@pytest.mark.parametrize("K", [256, 512, 1536, 2048])
@pytest.mark.parametrize("M", [47160, 33000, 45000])
def test_gemm_n512_large_m(dev, dtype, K, M):
    """The N = 512 text GEMMs at the headline's row counts (47,160 rows: the 192x256 ping-pong
    tiles, 492 tiles on 256 CUs) vs a torch fp32 reference: EPI_NONE (the input-grad GEMMs) and
    the 16-bit residual epilogue (out_proj / c_proj forward); reruns bitwise equal."""
    Nn = 512
    g = torch.Generator(device="cpu").manual_seed(M + K)
    A = torch.randn(M, K, generator=g).to(dev).to(dtype)
    B = (torch.randn(Nn, K, generator=g) / math.sqrt(K)).to(dev).to(dtype)
    bias = torch.randn(Nn, generator=g).to(dev)
    res = torch.randn(M, Nn, generator=g).to(dev).to(dtype)
    ref = A.float() @ B.float().t()
    o1 = ops.gemm(A, B, N.EPI_NONE, dtype)
    o2 = ops.gemm(A, B, N.EPI_NONE, dtype)
    torch.cuda.synchronize()
    assert torch.equal(o1, o2)
    close(o1, ref, dtype, f"n512 none K{K}")
    r1 = ops.gemm(A, B, N.EPI_BIAS_RES, dtype, bias=bias, res=res)
    close(r1, ref + bias + res.float(), dtype, f"n512 res K{K}")


def test_split_pack_range_and_stride(dev):
    """clipk_split_pack enforces |W| < 65504 / SPLIT_SCALE itself (CLIPK_ERANGE for a larger or a
    non-finite value), and the CLIPK_F32S GEMMs refuse a B row stride other than K (the packed
    weight's rows are exactly K elements apart)."""
    lib = N.load()
    K, Nn = 64, 128
    ok = torch.full((Nn, K), 65504.0 / N.SPLIT_SCALE * 0.999, device=dev)
    out = torch.empty(Nn, K, dtype=torch.int32, device=dev)
    assert lib.clipk_split_pack(Nn, K, ops._p(ok), K, ops._p(out), ops._stream()) == 0
    for bad in (65504.0 / N.SPLIT_SCALE, float("inf"), float("nan")):
        w = torch.zeros(Nn, K, device=dev)
        w[Nn - 1, K - 1] = bad
        assert lib.clipk_split_pack(Nn, K, ops._p(w), K, ops._p(out), ops._stream()) == -5, bad
    a = torch.randn(16, K, device=dev)
    o = torch.empty(16, Nn, device=dev)
    common = (N.F32S, N.F32, N.EPI_NONE, 16, Nn, K, ops._p(a), K, ops._p(out))
    assert lib.clipk_gemm(*common, 2 * K, None, None, Nn, ops._p(o), Nn, None, None, 0, Nn, ops._stream()) == -2
    assert lib.clipk_gemm(*common, K, None, None, Nn, ops._p(o), Nn, None, None, 0, Nn, ops._stream()) == 0
    torch.cuda.synchronize()


@pytest.mark.parametrize("reduction", ["mean", "sum", "none"])
def test_focal_loss_reductions(dev, reduction):
    """MultiClassFocalLoss(reduction=...) (PromptSRC/trainers/coop.py:131-163): loss and
    d logits vs the reference's formula in torch fp32 autograd, for each reduction."""
    from fsp_amd.trainers.losses import MultiClassFocalLoss
    g = torch.Generator(device="cpu").manual_seed(5)
    logits = (torch.randn(6, 37, generator=g) * 3).to(dev)
    y = torch.randint(0, 37, (6,), generator=g).to(dev)
    alpha = (torch.rand(37, generator=g) + 0.5).tolist()
    up = torch.randn(6, generator=g).to(dev)  # upstream gradient for 'none'
    fl = MultiClassFocalLoss(alpha=alpha, gamma=2, reduction=reduction)
    x = logits.clone().requires_grad_(True)
    out = fl(x, y)
    (out * up).sum().backward() if reduction == "none" else out.backward()
    xr = logits.clone().requires_grad_(True)
    ce = F.cross_entropy(xr, y, reduction="none")
    pt = torch.exp(-ce)
    fr = torch.tensor(alpha, device=dev)[y] * (1 - pt) ** 2 * ce
    ref = fr.mean() if reduction == "mean" else fr.sum() if reduction == "sum" else fr
    (ref * up).sum().backward() if reduction == "none" else ref.backward()
    assert out.shape == ref.shape
    close(out.detach(), ref.detach(), torch.float32, f"focal {reduction}")
    close(x.grad, xr.grad, torch.float32, f"focal {reduction} grad")


@pytest.mark.parametrize("cfg", [1, 6])
@pytest.mark.parametrize("K", [64, 128, 192, 320])
def test_gemm_large_tiles_short_k(dev, cfg, K):
    """The 256- / 192-row tile main loops at 1-5 K tiles (prologue / drain edge cases)."""
    lib = N.load()
    M, Nn = 5000, 512
    g = torch.Generator(device="cpu").manual_seed(K + cfg)
    A = torch.randn(M, K, generator=g).to(dev).to(torch.float16)
    B = (torch.randn(Nn, K, generator=g) / math.sqrt(K)).to(dev).to(torch.float16)
    bias = torch.randn(Nn, generator=g).to(dev)
    res = torch.randn(M, Nn, generator=g).to(dev)
    ref = A.float() @ B.float().t()
    try:
        N.check(lib.clipk_gemm_set_config(cfg), "set_config")
        close(ops.gemm(A, B, N.EPI_NONE, torch.float16), ref, torch.float16, f"cfg{cfg} K{K} none")
        close(ops.gemm(A, B, N.EPI_BIAS_RES, torch.float32, bias=bias, res=res), ref + bias + res,
              torch.float16, f"cfg{cfg} K{K} res")
    finally:
        lib.clipk_gemm_set_config(-1)


@pytest.mark.parametrize("dtype", [torch.float16, torch.bfloat16, torch.float32])
@pytest.mark.parametrize("M,Nn,K,splits",[(1576, 768, 3072, 0), (1576, 768, 768, 3), (1576, 2304, 768, 2),
                                           (300, 256, 512, 3)])
def test_gemm_splitk(dev, dtype, M, Nn, K, splits):
    """Split-K (ViT at small batch) vs torch fp32, every epilogue; slice-order sum is
    deterministic (bitwise-equal reruns)."""
    g = torch.Generator(device="cpu").manual_seed(M + Nn + K)
    A = torch.randn(M, K, generator=g).to(dev).to(dtype)
    B = (torch.randn(Nn, K, generator=g) / math.sqrt(K)).to(dev).to(dtype)
    bias = torch.randn(Nn, generator=g).to(dev)
    res = torch.randn(M, Nn, generator=g).to(dev)
    if splits == 0:
        assert N.load().clipk_gemm_auto_splits(ops.DT[dtype], M, Nn, K) > 1
    # 16-bit K = 768 (12 K steps) stays unsplit: slices need >= 8 K steps
    assert N.load().clipk_gemm_auto_splits(ops.DT[torch.float16], 1576, 768, 768) == 1
    ref = A.float() @ B.float().t()
    o1 = ops.gemm_splitk(A, B, N.EPI_NONE, torch.float32, splits=splits)
    close(o1, ref, dtype, "splitk none")
    assert torch.equal(o1, ops.gemm_splitk(A, B, N.EPI_NONE, torch.float32, splits=splits))
    close(ops.gemm_splitk(A, B, N.EPI_BIAS_RES, torch.float32, bias=bias, res=res, splits=splits),
          ref + bias + res, dtype, "splitk res")
    odt = dtype if dtype != torch.float32 else torch.float32
    gq, hq = ops.gemm_splitk(A, B, N.EPI_BIAS_QGELU, odt, bias=bias, want_out2=True, splits=splits)
    hr = ref + bias
    close(hq, hr, dtype, "splitk qgelu.h")
    close(gq, hr * torch.sigmoid(1.702 * hr), dtype, "splitk qgelu.g")
    gd, dd = ops.gemm_splitk(A, B, N.EPI_BIAS_QGELU | N.QGELU_DERIV, odt, bias=bias, want_out2=True, splits=splits)
    sg = torch.sigmoid(1.702 * hr)
    assert torch.equal(gd, gq)
    close(dd, sg * (1 + 1.702 * hr * (1 - sg)), dtype, "splitk qgelu deriv")
    close(ops.gemm_splitk(A, B, N.EPI_BIAS, odt, bias=bias, splits=splits), hr, dtype, "splitk bias")


def prefix_case(G, C, P, H, max_q, seed):
    """Random shared-prefix packing: per-class q_len in [1, max_q], group stride R, and the
    host-side attention tiles (whole classes packed into <= 16-row windows)."""
    from fsp_amd.trainers.prompt_base import attention_tiles
    g = torch.Generator().manual_seed(seed)
    qlen = torch.randint(1, max_q + 1, (C,), generator=g)
    qlen[0] = max_q
    off = P + torch.cat([torch.zeros(1, dtype=torch.long), qlen.cumsum(0)[:-1]])
    R = int(P + qlen.sum())
    tiles, row_first = attention_tiles(off.numpy(), qlen.numpy(), R)
    return R, torch.from_numpy(tiles.reshape(-1).copy()), torch.from_numpy(row_first), off.tolist(), qlen.tolist(), g


def attn_prefix_ref(qkv, G, C, P, R, off, qlen, H):
    """Unpacked restatement: each class sequence = [prefix rows, own rows], causal; the
    prefix rows' outputs from the prefix alone. Gathers from qkv (autograd sums shares)."""
    W = H * 64
    out = [None] * (G * R)
    lse = [None] * (G * R)
    for g in range(G):
        base = g * R
        seqs = [list(range(base, base + P))] + [list(range(base, base + P)) + list(range(base + off[c], base + off[c] + qlen[c])) for c in range(C)]
        dst = [list(range(base, base + P))] + [list(range(base + off[c], base + off[c] + qlen[c])) for c in range(C)]
        for idx, d in zip(seqs, dst):
            x = qkv[idx].float().view(len(idx), 3, H, 64).permute(1, 2, 0, 3)
            s = x[0] @ x[1].transpose(-1, -2) / 8.0
            Lq = len(idx)
            s = s + torch.full((Lq, Lq), float("-inf"), device=qkv.device).triu(1)
            o = (torch.softmax(s, -1) @ x[2]).permute(1, 0, 2).reshape(Lq, W)
            l = torch.logsumexp(s, -1).t()
            for i, r in enumerate(d):
                out[r] = o[Lq - len(d) + i]
                lse[r] = l[Lq - len(d) + i]
    return torch.stack(out), torch.stack(lse)


@pytest.mark.parametrize("dtype,gdtype", [(torch.float16, torch.bfloat16), (torch.bfloat16, torch.bfloat16),
                                          (torch.float16, torch.float16), (torch.float32, torch.float32)])
@pytest.mark.parametrize("G,C,P,H,max_q", [(2, 37, 5, 8, 6), (1, 19, 16, 2, 7), (3, 16, 2, 4, 16), (2, 3, 9, 2, 1),
                                           (2, 53, 5, 2, 3), (1, 40, 3, 2, 9),
                                           # enough waves for the fp32 kernels' units per wave
                                           # (f32_uc) to leave their 4-unit floor
                                           (24, 300, 5, 8, 7)])
def test_attention_prefix_fwd_bwd(dev, dtype, gdtype, G, C, P, H, max_q):
    R, tiles, row_first, off, qlen, g = prefix_case(G, C, P, H, max_q, seed=G * 100 + C + P)
    W = H * 64
    qkv = torch.randn(G * R, 3 * W, generator=g).to(dev).to(dtype)
    tiles, row_first = tiles.to(dev), row_first.to(dev)
    o, lse = ops.attention_prefix(qkv, G, P, R, tiles, row_first, H, lse=True)
    q32 = qkv.float().requires_grad_(True)
    ro, rl = attn_prefix_ref(q32, G, C, P, R, off, qlen, H)
    close(o, ro, dtype, "prefix attn out")
    close(lse, rl, torch.float16 if dtype != torch.float32 else dtype, "prefix attn lse")
    dout = torch.randn(G * R, W, generator=g).to(dev).to(gdtype)
    (ro * dout.float()).sum().backward()
    dq = ops.attention_prefix_bwd(qkv, o, dout, lse, G, P, R, tiles, row_first, H, gdtype)
    ref = q32.grad
    for part, sl in (("dq", slice(0, W)), ("dk", slice(W, 2 * W)), ("dv", slice(2 * W, 3 * W))):
        close(dq[:, sl], ref[:, sl], gdtype if dtype != torch.float32 else dtype, f"prefix attn {part}")


@pytest.mark.parametrize("dtype,gdtype", [(torch.float16, torch.float16), (torch.bfloat16, torch.bfloat16),
                                          (torch.float32, torch.float32)])
@pytest.mark.parametrize("G,C,P,H,max_q", [(3, 37, 5, 8, 6), (2, 19, 16, 2, 7), (24, 300, 5, 8, 7)])
def test_attention_prefix_cls_group0(dev, dtype, gdtype, G, C, P, H, max_q):
    """CLIPK_PREFIX_CLS_GROUP0 (the text encoder's shared layer 0): with every group's class rows
    of q|k|v read from group 0, forward and backward are bitwise the plain calls on a qkv whose
    class rows were copied into every group -- here the other groups' class rows hold NaN, so a
    read of them would show."""
    R, tiles, row_first, off, qlen, g = prefix_case(G, C, P, H, max_q, seed=G * 100 + C + P + 7)
    W = H * 64
    qkv = torch.randn(G * R, 3 * W, generator=g).to(dev).to(dtype)
    for gg in range(1, G):
        qkv[gg * R + P:(gg + 1) * R] = qkv[P:R]
    hole = qkv.clone()
    for gg in range(1, G):
        hole[gg * R + P:(gg + 1) * R] = float("nan")
    tiles, row_first = tiles.to(dev), row_first.to(dev)
    o, lse = ops.attention_prefix(qkv, G, P, R, tiles, row_first, H, lse=True)
    o2, lse2 = ops.attention_prefix(hole, G, P, R, tiles, row_first, H, lse=True, flags=N.PREFIX_CLS_GROUP0)
    assert torch.equal(o, o2) and torch.equal(lse, lse2)
    dout = torch.randn(G * R, W, generator=g).to(dev).to(gdtype)
    d1 = ops.attention_prefix_bwd(qkv, o, dout, lse, G, P, R, tiles, row_first, H, gdtype)
    d2 = ops.attention_prefix_bwd(hole, o, dout, lse, G, P, R, tiles, row_first, H, gdtype, flags=N.PREFIX_CLS_GROUP0)
    assert torch.equal(d1, d2)


@pytest.mark.parametrize("knobs", [
    {"CLIPK_PREFIX_LDS": "0"},
    {"CLIPK_PREFIX_LDS": "3", "CLIPK_PREFIX_LDS_WPB": "1"},
    {"CLIPK_PREFIX_LDS": "2", "CLIPK_PREFIX_LDS_WPB": "2", "CLIPK_PREFIX_FWD_CHUNK": "1",
     "CLIPK_PREFIX_BWD_CHUNK": "3"},
])
def test_attention_prefix_kernel_variants(knobs):
    """The other shared-prefix attention variants -- the register-operand kernels, a 3-slot
    LDS ring, 1- and 2-wave blocks, 1- and 3-tile chunks -- through the same cases, in a child
    process (the knobs are read once per process)."""
    env = dict(os.environ, **knobs)
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-p", "no:cacheprovider", os.path.abspath(__file__),
                        "-k", "test_attention_prefix_fwd_bwd"], env=env, capture_output=True, text=True, timeout=300,
                       cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]
    assert "28 passed" in r.stdout, r.stdout[-500:]  # 4 dtype pairs x 7 shapes


def test_prompt_rows_and_ctx_grad_rows(dev):
    """Packed assembly + slot-list ctx grad against torch on the same tables."""
    from fsp_amd.trainers._fns import prompt_layout
    from fsp_amd.trainers.prompt_base import shared_prefix_tables
    C, n_ctx, W, G = 9, 4, 128, 3
    name_lens = [1, 2, 3, 1, 4, 2, 5, 1, 2]
    eot = [1 + n_ctx + nl + 1 for nl in name_lens]
    src, cpos, L = prompt_layout(C, n_ctx, name_lens, "end", eot)
    pk = shared_prefix_tables(src, cpos, eot, n_ctx, csc=False)
    g = torch.Generator().manual_seed(3)
    emb = torch.randn(C, 77, W, generator=g).to(dev)
    ctx = torch.randn(n_ctx, W, generator=g).to(dev)
    bias = torch.randn(G, W, generator=g).to(dev)
    pos = torch.randn(77, W, generator=g).to(dev)
    t = lambda a: torch.from_numpy(a).to(dev)
    R = pk["R"]
    x0 = ops.prompt_assemble_rows(G, R, C, L, t(pk["row_tab"]), t(src), emb, ctx, 0, 0, bias, pos)
    ref = torch.empty(G * R, W, device=dev)
    for gg in range(G):
        for r in range(R):
            c, tt = divmod(int(pk["row_tab"][r]), L)
            m = int(src[c, tt])
            ref[gg * R + r] = (emb[c, m] if m >= 0 else ctx[-1 - m] + bias[gg]) + pos[tt]
    torch.testing.assert_close(x0, ref, rtol=0, atol=1e-6)
    dx = torch.randn(G * R, W, generator=g).to(dev)
    d = ops.ctx_grad_rows(G, R, W, n_ctx, t(pk["slot_ptr"]), t(pk["slot_rows"]), dx)
    ctx_r = ctx.clone().requires_grad_(True)
    bias_r = bias.clone().requires_grad_(True)
    rows = []
    for gg in range(G):
        for r in range(R):
            c, tt = divmod(int(pk["row_tab"][r]), L)
            m = int(src[c, tt])
            rows.append((ctx_r[-1 - m] + bias_r[gg]) if m < 0 else torch.zeros(W, device=dev))
    (torch.stack(rows) * dx).sum().backward()
    d = d.view(G, n_ctx, W)
    torch.testing.assert_close(d.sum(0), ctx_r.grad, rtol=1e-5, atol=1e-4)
    torch.testing.assert_close(d.sum(1), bias_r.grad, rtol=1e-5, atol=1e-4)
    # the same two sums in one launch (clipk_ctx_bias_grad_rows): d ctx in g order, d bias in k order
    dctx, dbias = ops.ctx_bias_grad_rows(G, R, W, n_ctx, t(pk["slot_ptr"]), t(pk["slot_rows"]), dx)
    sg = d[0].clone()
    for gg in range(1, G):
        sg = sg + d[gg]
    sk = d[:, 0].clone()
    for k in range(1, n_ctx):
        sk = sk + d[:, k]
    assert torch.equal(dctx, sg) and torch.equal(dbias, sk)
    dctx2, none = ops.ctx_bias_grad_rows(G, R, W, n_ctx, t(pk["slot_ptr"]), t(pk["slot_rows"]), dx, bias=False)
    assert none is None and torch.equal(dctx2, dctx)
