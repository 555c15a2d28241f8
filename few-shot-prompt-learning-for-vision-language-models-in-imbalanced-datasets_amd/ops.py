"""Tensor-level wrappers over the C-ABI: torch tensors in, device pointers + the
current HIP stream out. torch is plumbing here (allocation, streams); every op's
arithmetic runs in libclipk.so. Inputs are validated on the host and errors map to
``ClipkError`` (RuntimeError) naming the op and status, mirroring the reference's
Python exceptions at module level.
"""
from __future__ import annotations

import ctypes

import torch

from . import _native as N

DT = {torch.float32: N.F32, torch.float16: N.F16, torch.bfloat16: N.BF16}


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _p(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _need(t, name, dtype=None, cuda=True):
    if t is None:
        raise N.ClipkError(f"{name} is required")
    if cuda and not t.is_cuda:
        raise N.ClipkError(f"{name} must be a CUDA(HIP) tensor; no CPU path exists")
    if dtype is not None and t.dtype != dtype:
        raise N.ClipkError(f"{name} must be {dtype}, got {t.dtype}")
    if not t.is_contiguous():
        raise N.ClipkError(f"{name} must be contiguous")
    return t


def split_pack(w):
    """clipk_split_pack: fp32 weight [N, K] -> its split-fp16 packing for PREC fp32s
    (SPLIT_SCALE * w as fp16 hi + lo parts, 4 bytes per element; int32 storage [N, K])."""
    _need(w, "W", torch.float32)
    n, k = w.shape
    if k % 32:
        raise N.ClipkError(f"split_pack needs K % 32 == 0, got {k}")
    out = torch.empty(n, k, dtype=torch.int32, device=w.device)
    # the library checks |W| < 65504 / SPLIT_SCALE itself (CLIPK_ERANGE)
    N.call("clipk_split_pack", n, k, _p(w), k, _p(out), _stream())
    return out


def split_lo_zero(packed) -> bool:
    """clipk_split_lo_zero: whether every lo part of a split_pack(...) weight is zero (the weight
    is fp16-valued, so split_hi16 compacts it for CLIPK_F32S16). Synchronises the stream."""
    _need(packed, "packed", torch.int32)
    n, k = packed.shape
    res = ctypes.c_int(-1)
    N.call("clipk_split_lo_zero", n, k, _p(packed), ctypes.byref(res), _stream())
    if res.value not in (0, 1):
        raise N.ClipkError(f"clipk_split_lo_zero: no answer ({res.value})")
    return res.value == 1


def split_hi16(packed):
    """clipk_split_hi16: the CLIPK_F32S16 B operand of an fp16-valued split_pack(...) weight -- fp16
    [N, K] = SPLIT_SCALE * W exactly (2 B per element). Raises (CLIPK_ERANGE) when W is not
    fp16-valued. Synchronises the stream."""
    _need(packed, "packed", torch.int32)
    n, k = packed.shape
    out = torch.empty(n, k, dtype=torch.float16, device=packed.device)
    N.call("clipk_split_hi16", n, k, _p(packed), _p(out), _stream())
    return out


def _split_kind(a, b):
    """The GEMM input type for (a, b): PREC fp32s when a is fp32 and b a split weight -- int32
    split_pack(...) (CLIPK_F32S) or fp16 split_hi16(...) (CLIPK_F32S16) -- else None."""
    if a.dtype != torch.float32:
        return None
    return {torch.int32: N.F32S, torch.float16: N.F32S16}.get(b.dtype)


def gemm(a, b, epi=N.EPI_NONE, out_dtype=torch.float32, bias=None, res=None, aux=None,
         want_out2=False, out=None):
    """out[M,N] = epi(a[M,K] @ b[N,K]^T); returns out (and out2 for EPI_BIAS_QGELU). With a
    fp32 and b a split weight: the fp32-class split-fp16 GEMM (b int32 split_pack(...):
    CLIPK_F32S; b fp16 split_hi16(...) of an fp16-valued weight: CLIPK_F32S16)."""
    _need(a, "A")
    split = _split_kind(a, b)
    _need(b, "B", b.dtype if split is not None else a.dtype)
    M, K = a.shape
    Nn = b.shape[0]
    if b.shape[1] != K:
        raise N.ClipkError(f"gemm K mismatch {tuple(a.shape)} x {tuple(b.shape)}^T")
    if out is None:
        out = torch.empty(M, Nn, device=a.device, dtype=out_dtype)
    out2 = torch.empty_like(out) if want_out2 else None
    if bias is not None:
        _need(bias, "bias", torch.float32)
    if res is not None:
        _need(res, "res", torch.float32 if out.dtype == torch.float32 else out.dtype)
    if aux is not None:
        _need(aux, "aux")
    args = (split if split is not None else DT[a.dtype], DT[out.dtype], epi, M, Nn, K, _p(a), K, _p(b), K, _p(bias),
            _p(res), Nn, _p(out), Nn, _p(out2), _p(aux), DT[aux.dtype] if aux is not None else 0, Nn)
    N.call("clipk_gemm", *args, _stream())
    return (out, out2) if want_out2 else out


def gemm_ln(a, b, epi, bias, stats=None, res=None, colsum=None, rnb=None, want_out2=False):
    """clipk_gemm_ln (include/clipk.h): 16-bit a[M,K] @ b[N,K]^T with the LayerNorm fold.
    Producer (EPI_BIAS_RES, colsum None): the statistics partials of the output are written to
    stats (fp32 [M, N/64, 2]). Fold (EPI_BIAS / EPI_BIAS_QGELU): a is the LayerNorm input x with
    per-row rnb = (rstd, -rstd * mean) (ln_stats_merge of its partials), b = W diag(gamma),
    bias = b + W beta, colsum = row sums of b. Output in a's dtype. PREC fp32s: a fp32 and b a
    split weight as in gemm (colsum summed over the packed value, see clip.model.ln_fold_weights)."""
    _need(a, "A")
    split = _split_kind(a, b)
    _need(b, "B", b.dtype if split is not None else a.dtype)
    M, K = a.shape
    Nn = b.shape[0]
    out = torch.empty(M, Nn, device=a.device, dtype=a.dtype)
    out2 = torch.empty_like(out) if want_out2 else None
    _need(bias, "bias", torch.float32)
    for t, nm in ((stats, "stats"), (colsum, "colsum"), (rnb, "rnb")):
        if t is not None:
            _need(t, nm, torch.float32)
    if res is not None:
        _need(res, "res", a.dtype)
    N.call("clipk_gemm_ln", split if split is not None else DT[a.dtype], epi, M, Nn, K, _p(a), K, _p(b), K, _p(bias),
           _p(res), Nn, _p(out), Nn, _p(out2), _p(stats), _p(colsum), _p(rnb), _stream())
    return (out, out2) if want_out2 else out


def gemm_ln_gamma(a, b, epi, bias, colsum, rnb, gamma, want_out2=False):
    """clipk_gemm_ln_gamma (PREC fp32s): the LayerNorm fold with gamma applied to A: a fp32 x,
    b = W itself as a split weight (int32 split_pack(W): CLIPK_F32S; fp16 split_hi16(...):
    CLIPK_F32S16), colsum = rowsums of W diag(gamma), bias = b + W beta, rnb = (rstd, -rstd *
    mean) per row."""
    _need(a, "A", torch.float32)
    split = _split_kind(a, b)
    if split is None:
        raise N.ClipkError(f"gemm_ln_gamma: B must be a split weight (int32 / fp16), got {b.dtype}")
    _need(b, "B", b.dtype)
    M, K = a.shape
    Nn = b.shape[0]
    out = torch.empty(M, Nn, device=a.device, dtype=torch.float32)
    out2 = torch.empty_like(out) if want_out2 else None
    for t, nm in ((bias, "bias"), (colsum, "colsum"), (rnb, "rnb"), (gamma, "gamma")):
        _need(t, nm, torch.float32)
    N.call("clipk_gemm_ln_gamma", split, epi, M, Nn, K, _p(a), K, _p(b), K, _p(bias),
           _p(out), Nn, _p(out2), _p(colsum), _p(rnb), _p(gamma), _stream())
    return (out, out2) if want_out2 else out


def gemm_ln_stats_split(a, b, epi, bias, stats, res, gamma):
    """clipk_gemm_ln_stats_split (PREC fp32s, split mode 2): the LayerNorm-statistics producer
    (EPI_BIAS_RES [| A_SPLIT], b a split_hi16 weight) that also writes the next fold's pre-split A,
    split(out * gamma). Returns (out fp32 [M, N], out2 [M, N] fp32 storage of fp16 parts)."""
    _need(a, "A", torch.float32)
    _need(b, "B", torch.float16)
    M, K = a.shape
    Nn = b.shape[0]
    out = torch.empty(M, Nn, device=a.device, dtype=torch.float32)
    out2 = torch.empty_like(out)
    for t, nm in ((bias, "bias"), (stats, "stats"), (res, "res"), (gamma, "gamma")):
        _need(t, nm, torch.float32)
    N.call("clipk_gemm_ln_stats_split", N.F32S16, epi, M, Nn, K, _p(a), K, _p(b), K, _p(bias), _p(res), Nn,
           _p(out), Nn, _p(stats), _p(gamma), _p(out2), _stream())
    return out, out2


def gemm_ln_merge(a, b, epi, bias, stats, colsum, want_out2=False):
    """clipk_gemm_ln_merge: ln_stats_merge(stats, K) then the fold gemm_ln(a, b, epi, bias,
    colsum=colsum, rnb=...), as one launch where the library covers the shape. Returns
    (out[, out2], mean, rstd, rnb); 16-bit a."""
    _need(a, "A")
    _need(b, "B", a.dtype)
    _need(stats, "stats", torch.float32)
    _need(colsum, "colsum", torch.float32)
    _need(bias, "bias", torch.float32)
    M, K = a.shape
    Nn = b.shape[0]
    out = torch.empty(M, Nn, device=a.device, dtype=a.dtype)
    out2 = torch.empty_like(out) if want_out2 else None
    mean = torch.empty(M, device=a.device, dtype=torch.float32)
    rstd = torch.empty_like(mean)
    rnb = torch.empty(M, 2, device=a.device, dtype=torch.float32)
    N.call("clipk_gemm_ln_merge", DT[a.dtype], epi, M, Nn, K, _p(a), K, _p(b), K, _p(bias), _p(out), Nn, _p(out2),
           _p(stats), _p(colsum), _p(mean), _p(rstd), _p(rnb), _stream())
    return ((out, out2) if want_out2 else (out,)) + (mean, rstd, rnb)


def ln_stats_merge(stats, width):
    """clipk_ln_stats_merge: [M, width/64, 2] partials -> (mean, rstd, rnb): fp32 [M], [M], [M, 2]
    with rnb = (rstd, -rstd * mean)."""
    _need(stats, "stats", torch.float32)
    M = stats.shape[0]
    mean = torch.empty(M, device=stats.device, dtype=torch.float32)
    rstd = torch.empty_like(mean)
    rnb = torch.empty(M, 2, device=stats.device, dtype=torch.float32)
    N.call("clipk_ln_stats_merge", M, width, _p(stats), _p(mean), _p(rstd), _p(rnb), _stream())
    return mean, rstd, rnb


def gemm_splitk(a, b, epi=N.EPI_NONE, out_dtype=torch.float32, bias=None, res=None, want_out2=False,
                splits=0):
    """Split-K form of gemm (fp32 partials in a workspace, deterministic slice-order sum);
    splits <= 0 picks the library's choice for the shape."""
    _need(a, "A")
    split = _split_kind(a, b)
    _need(b, "B", b.dtype if split is not None else a.dtype)
    ind = split if split is not None else DT[a.dtype]
    M, K = a.shape
    Nn = b.shape[0]
    if splits <= 0:
        splits = N.load().clipk_gemm_auto_splits(ind, M, Nn, K)
    out = torch.empty(M, Nn, device=a.device, dtype=out_dtype)
    out2 = torch.empty_like(out) if want_out2 else None
    ws = torch.empty(max(N.load().clipk_gemm_splitk_ws_bytes(M, Nn, splits), 1), dtype=torch.uint8,
                     device=a.device)
    N.call("clipk_gemm_splitk", ind, DT[out_dtype], epi, M, Nn, K, _p(a), K, _p(b), K, _p(bias),
           _p(res), Nn, _p(out), Nn, _p(out2), splits, _p(ws), ws.numel(), _stream())
    return (out, out2) if want_out2 else out


def layernorm(x, w, b, out_dtype=torch.float32, rows=None, stats=False):
    """LayerNorm over the last dim of x [R, W] (fp32 or 16-bit; optionally on gathered rows)."""
    _need(x, "x")
    R, W = x.shape
    n = R if rows is None else rows.numel()
    out = torch.empty(n, W, device=x.device, dtype=out_dtype)
    mean = torch.empty(n, device=x.device) if stats else None
    rstd = torch.empty(n, device=x.device) if stats else None
    if rows is not None:
        _need(rows, "rows", torch.int32)
    N.call("clipk_layernorm_fwd_x", DT[x.dtype], DT[out_dtype], n, W, _p(x), W, _p(rows), _p(w), _p(b), _p(out),
           W, _p(mean), _p(rstd), _stream())
    return (out, mean, rstd) if stats else out


def layernorm_bwd(dy, x, w, mean, rstd, dres=None, lp_dtype=None):
    """LayerNorm input-grad (+ dres) into fp32 dx and, with lp_dtype, a second copy dx_lp; lp_dtype
    "split": dx_lp in the pre-split operand form (CLIPK_A_SPLIT; fp32 storage of fp16 parts)."""
    _need(dy, "dy")
    R, W = dy.shape
    dx = torch.empty(R, W, device=dy.device, dtype=torch.float32)
    split = lp_dtype == "split"
    lp = (torch.empty(R, W, device=dy.device, dtype=torch.float32 if split else lp_dtype)
          if lp_dtype is not None else None)
    lpd = N.F32S if split else (DT[lp_dtype] if lp_dtype is not None else 0)
    _need(x, "x")
    N.call("clipk_layernorm_bwd_x", DT[x.dtype], DT[dy.dtype], R, W, _p(dy), W, _p(x), W, None, _p(w), _p(mean),
           _p(rstd), _p(dres), W, _p(dx), _p(lp), lpd, None, W, _stream())
    return (dx, lp) if lp is not None else dx


def layernorm_bwd_lp_(dy, x, w, mean, rstd, dres_lp, dx=None):
    """16-bit residual-gradient stream: dres_lp <- LN-input-grad(dy) + dres_lp, in place (the
    dtype of dres_lp); also into fp32 dx when given. Returns dres_lp."""
    _need(dy, "dy")
    _need(x, "x")
    _need(dres_lp, "dres_lp")
    R, W = dy.shape
    N.call("clipk_layernorm_bwd_x2", DT[x.dtype], DT[dy.dtype], R, W, _p(dy), W, _p(x), W, None, _p(w), _p(mean),
           _p(rstd), _p(dres_lp), DT[dres_lp.dtype], W, _p(dx), _p(dres_lp), DT[dres_lp.dtype], None, W, _stream())
    return dres_lp


def attention(qkv, nseq, L, heads, causal, lse=False):
    _need(qkv, "qkv")
    W = heads * 64
    out = torch.empty(nseq * L, W, device=qkv.device, dtype=qkv.dtype)
    l = torch.empty(nseq * L, heads, device=qkv.device) if lse else None
    N.call("clipk_attention_fwd", DT[qkv.dtype], nseq, L, heads, int(causal), _p(qkv), 3 * W, _p(out),
           W, _p(l), _stream())
    return (out, l) if lse else out


def attention_bwd(qkv, o, dout, lse, nseq, L, heads, causal, grad_dtype):
    W = heads * 64
    dqkv = torch.empty(nseq * L, 3 * W, device=qkv.device, dtype=grad_dtype)
    N.call("clipk_attention_bwd", DT[qkv.dtype], DT[grad_dtype], nseq, L, heads, int(causal), _p(qkv),
           3 * W, _p(o), W, _p(dout), W, _p(lse), _p(dqkv), 3 * W, _stream())
    return dqkv


def im2col(img, patch, Kp, out_dtype):
    _need(img, "image", torch.float32)
    B, _, R, _ = img.shape
    G = R // patch
    out = torch.empty(B * G * G, Kp, device=img.device, dtype=out_dtype)
    N.call("clipk_im2col", DT[out_dtype], B, R, patch, Kp, _p(img), _p(out), _stream())
    return out


def prompt_assemble(B, C, L, src_map, emb, ctx, ctx_sb, ctx_sc, bias, pos):
    W = emb.shape[-1]
    x0 = torch.empty(B * C * L, W, device=emb.device, dtype=torch.float32)
    N.call("clipk_prompt_assemble", B, C, L, W, _p(src_map), _p(emb), _p(ctx), ctx_sb, ctx_sc, _p(bias),
           _p(pos), _p(x0), _stream())
    return x0


def prompt_assemble_rows(G, R, C, L, row_tab, src_map, emb, ctx, ctx_sg, ctx_sc, bias, pos):
    W = emb.shape[-1]
    x0 = torch.empty(G * R, W, device=emb.device, dtype=torch.float32)
    N.call("clipk_prompt_assemble_rows", G, R, C, L, W, _p(row_tab), _p(src_map), _p(emb), _p(ctx), ctx_sg,
           ctx_sc, _p(bias), _p(pos), _p(x0), _stream())
    return x0


def ctx_bias_grad_rows(G, R, W, n_ctx, slot_ptr, slot_rows, dx0, bias=True):
    """clipk_ctx_bias_grad_rows: (dctx [n_ctx, W] summed over the G groups, dbias [G, W] summed
    over the slots, or None)."""
    dctx = torch.empty(n_ctx, W, device=dx0.device, dtype=torch.float32)
    dbias = torch.empty(G, W, device=dx0.device, dtype=torch.float32) if bias else None
    N.call("clipk_ctx_bias_grad_rows", G, R, W, n_ctx, _p(slot_ptr), _p(slot_rows), _p(dx0), _p(dctx), _p(dbias),
           _stream())
    return dctx, dbias


def ctx_grad_rows(G, R, W, n_ctx, slot_ptr, slot_rows, dx0):
    d = torch.empty(G * n_ctx, W, device=dx0.device, dtype=torch.float32)
    N.call("clipk_ctx_grad_rows", G, R, W, n_ctx, _p(slot_ptr), _p(slot_rows), _p(dx0), _p(d), _stream())
    return d


def attention_prefix(qkv, G, P, R, tiles, row_first, heads, lse=False, flags=0):
    """Shared-prefix packed causal attention (clipk_attention_prefix_fwd_ex); tiles int32
    [ntiles*2] (first row, rows), row_first int32 [R]; flags N.PREFIX_CLS_GROUP0: class rows'
    q|k|v read from group 0."""
    _need(qkv, "qkv")
    _need(tiles, "tiles", torch.int32)
    _need(row_first, "row_first", torch.int32)
    W = heads * 64
    out = torch.zeros(G * R, W, device=qkv.device, dtype=qkv.dtype)
    l = torch.zeros(G * R, heads, device=qkv.device) if lse else None
    N.call("clipk_attention_prefix_fwd_ex", DT[qkv.dtype], G, P, R, tiles.numel() // 2, _p(tiles), _p(row_first),
           heads, _p(qkv), 3 * W, _p(out), W, _p(l), int(flags), _stream())
    return (out, l) if lse else out


def attention_prefix_bwd(qkv, o, dout, lse, G, P, R, tiles, row_first, heads, grad_dtype, split=False, flags=0):
    """split (fp32 qkv / dout / grad_dtype): dq|dk|dv in the pre-split operand form of CLIPK_A_SPLIT
    (grad dtype CLIPK_F32S), viewed as fp32 [G*R, 3W]."""
    W = heads * 64
    nt = tiles.numel() // 2
    dqkv = torch.zeros(G * R, 3 * W, device=qkv.device, dtype=grad_dtype)
    nb = N.load().clipk_attention_prefix_ws_bytes(G, nt, heads)
    ws = torch.empty(nb, dtype=torch.uint8, device=qkv.device)
    gdt = N.F32S if split else DT[grad_dtype]
    N.call("clipk_attention_prefix_bwd_ex", DT[qkv.dtype], gdt, G, P, R, nt, _p(tiles), _p(row_first),
           heads, _p(qkv), 3 * W, _p(o), W, _p(dout), W, _p(lse), _p(dqkv), 3 * W, _p(ws), nb, int(flags), _stream())
    return dqkv


def ctx_grad(B, C, L, W, n_ctx, csc, ctx_pos, dx0):
    outs = (B * C if csc else B) * n_ctx
    d = torch.empty(outs, W, device=dx0.device, dtype=torch.float32)
    N.call("clipk_ctx_grad", B, C, L, W, n_ctx, int(csc), _p(ctx_pos), _p(dx0), _p(d), _stream())
    return d


def cosine_logits(imf, txt, scale, per_image, C):
    B, E = imf.shape
    logits = torch.empty(B, C, device=imf.device)
    inv_t = torch.empty(txt.shape[0], device=imf.device)
    inv_i = torch.empty(B, device=imf.device)
    N.call("clipk_cosine_logits_fwd", B, C, E, int(per_image), float(scale), _p(imf), _p(txt),
           _p(logits), _p(inv_t), _p(inv_i), _stream())
    return logits, inv_t, inv_i


def cosine_logits_bwd(imf, txt, inv_t, inv_i, dlogits, scale, per_image):
    B, C = dlogits.shape
    E = imf.shape[1]
    dtxt = torch.empty_like(txt)
    N.call("clipk_cosine_logits_bwd", B, C, E, int(per_image), float(scale), _p(imf), _p(txt),
           _p(inv_t), _p(inv_i), _p(dlogits.contiguous()), _p(dtxt), _stream())
    return dtxt


def ce_loss(logits, labels, alpha=None, gamma=2.0, focal=False, grad=True, grad_scale=None):
    """Per-row CE / focal loss [B] and dlogits = grad_scale * d(row loss)/d logits (default
    grad_scale 1/B: the gradient of the mean)."""
    _need(logits, "logits", torch.float32)
    _need(labels, "labels", torch.int64)
    B, C = logits.shape
    if labels.shape != (B,):
        raise N.ClipkError(f"labels must be [{B}], got {tuple(labels.shape)}")
    if alpha is not None:
        _need(alpha, "alpha", torch.float32)
        if alpha.numel() < C:
            raise N.ClipkError(f"alpha must hold {C} class weights, got {alpha.numel()}")
    row = torch.empty(B, device=logits.device)
    dl = torch.empty_like(logits) if grad else None
    N.call("clipk_ce_loss", B, C, _p(logits), _p(labels), _p(alpha), float(gamma), int(focal),
           float(1.0 / B if grad_scale is None else grad_scale), _p(row), _p(dl), _stream())
    return row, dl


def meta_net(x, w1, b1, w2, b2, normalize=False):
    """(h, y); normalize: the Meta-Net on x / |x| (clipk_meta_net_fwd_norm) -> (xn, h, y)."""
    B, V = x.shape
    Hd, Wd = w1.shape[0], w2.shape[0]
    h = torch.empty(B, Hd, device=x.device)
    y = torch.empty(B, Wd, device=x.device)
    if normalize:
        xn = torch.empty(B, V, device=x.device)
        N.call("clipk_meta_net_fwd_norm", B, V, Hd, Wd, _p(x), _p(w1), _p(b1), _p(w2), _p(b2), _p(xn), _p(h),
               _p(y), _stream())
        return xn, h, y
    N.call("clipk_meta_net_fwd", B, V, Hd, Wd, _p(x), _p(w1), _p(b1), _p(w2), _p(b2), _p(h), _p(y),
           _stream())
    return h, y


def ce_loss_reduce(logits, labels, alpha=None, gamma=2.0, focal=False, grad=True, reduction="mean"):
    """clipk_ce_loss_reduce: (loss [] = mean / sum of the row losses, dlogits = d loss / d logits)
    in one launch."""
    _need(logits, "logits", torch.float32)
    _need(labels, "labels", torch.int64)
    B, C = logits.shape
    if labels.shape != (B,):
        raise N.ClipkError(f"labels must be [{B}], got {tuple(labels.shape)}")
    if alpha is not None:
        _need(alpha, "alpha", torch.float32)
        if alpha.numel() < C:
            raise N.ClipkError(f"alpha must hold {C} class weights, got {alpha.numel()}")
    red = {"mean": 1, "sum": 2}[reduction]
    row = torch.empty(B, device=logits.device)
    loss = torch.empty((), device=logits.device)
    dl = torch.empty_like(logits) if grad else None
    N.call("clipk_ce_loss_reduce", B, C, _p(logits), _p(labels), _p(alpha), float(gamma), int(focal),
           1.0 / B if reduction == "mean" else 1.0, red, _p(row), _p(loss), _p(dl), _stream())
    return loss, dl


def status_take(flags, host_word):
    """clipk_status_take: flags -> host_word (pinned int32), flags cleared (stream-ordered)."""
    N.call("clipk_status_take", _p(flags), _p(host_word), _stream())


def meta_net_bwd(x, h, w2, dy, V, Hd, Wd):
    B = x.shape[0]
    dw1 = torch.empty(Hd, V, device=x.device)
    db1 = torch.empty(Hd, device=x.device)
    dw2 = torch.empty(Wd, Hd, device=x.device)
    db2 = torch.empty(Wd, device=x.device)
    dh = torch.empty(B, Hd, device=x.device)
    N.call("clipk_meta_net_bwd", B, V, Hd, Wd, _p(x), _p(h), _p(w2), _p(dy.contiguous()), _p(dw1),
           _p(db1), _p(dw2), _p(db2), _p(dh), _stream())
    return dw1, db1, dw2, db2


def sgd_step(p, g, buf, lr, momentum, weight_decay, has_buf):
    N.call("clipk_sgd_step", p.numel(), _p(p), _p(g), _p(buf), float(lr), float(momentum),
           float(weight_decay), int(has_buf), _stream())


def sgd_step_multi(ps, gs, bufs, lr, momentum, weight_decay, has_bufs, grad_scale=1.0, guard=None):
    """clipk_sgd_step_multi(_scaled / _if): one launch per 16 tensors (fp32, contiguous, on one
    device); grad_scale multiplies every gradient (1.0: the unscaled entry point); guard = (int32
    device flags, mask): the update is skipped on the device when flags[0] & mask."""
    import ctypes
    for i in range(0, len(ps), 16):
        P_, G_, B_ = ps[i:i + 16], gs[i:i + 16], bufs[i:i + 16]
        c = len(P_)
        VP = ctypes.c_void_p * c
        args = (c, VP(*[t.data_ptr() for t in P_]), VP(*[t.data_ptr() for t in G_]),
                VP(*[t.data_ptr() for t in B_]), (ctypes.c_long * c)(*[t.numel() for t in P_]),
                (ctypes.c_int * c)(*[int(h) for h in has_bufs[i:i + 16]]), float(lr), float(momentum),
                float(weight_decay))
        if guard is not None:
            N.call("clipk_sgd_step_multi_if", *args, float(grad_scale), _p(guard[0]), int(guard[1]), _stream())
        elif grad_scale == 1.0:
            N.call("clipk_sgd_step_multi", *args, _stream())
        else:
            N.call("clipk_sgd_step_multi_scaled", *args, float(grad_scale), _stream())


def cast(x, dtype):
    y = torch.empty(x.shape, device=x.device, dtype=dtype)
    N.call("clipk_cast", DT[dtype], x.numel(), _p(x.contiguous()), _p(y), _stream())
    return y


def rows_inject(src, rows, dst, n_per):
    """dst[rows[p*n_per + i]] = src[p] (deep prompts: the rows a layer's learnable tokens
    replace, model.py:229-256); src fp32 [n_ctx, W], dst [*, W] any dtype, in place."""
    _need(src, "prompt rows", torch.float32)
    _need(rows, "row table", torch.int32)
    _need(dst, "destination")
    n_ctx, W = src.shape
    N.call("clipk_rows_inject", DT[dst.dtype], n_ctx, n_per, W, _p(src), _p(rows), _p(dst), dst.shape[-1], _stream())
    return dst


def rows_collect(src, rows, n_ctx, n_per, out=None, zero_src=True, src2=None):
    """out[p] = sum_i src[rows[p*n_per + i]] (fixed order); those rows of src (and src2) zeroed."""
    _need(src, "gradient rows")
    _need(rows, "row table", torch.int32)
    W = src.shape[-1]
    acc = out is not None
    if out is None:
        out = torch.empty(n_ctx, W, device=src.device, dtype=torch.float32)
    N.call("clipk_rows_collect", DT[src.dtype], n_ctx, n_per, W, _p(src), W, _p(src2),
           DT[src2.dtype] if src2 is not None else 0, W if src2 is not None else 0, _p(rows), _p(out), int(acc),
           int(zero_src), _stream())
    return out
