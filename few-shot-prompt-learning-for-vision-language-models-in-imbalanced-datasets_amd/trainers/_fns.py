"""Autograd Functions wiring the native kernels into the prompt learners, plus the
host-side prompt layout tables. Every forward/backward body is a libclipk.so call;
torch only allocates and sums a handful of [B, n_ctx, W] values.
"""
from __future__ import annotations

import numpy as np
import torch

from .. import ops


def prompt_layout(n_cls, n_ctx, name_lens, position, eot, truncate=True):
    """Token-slot tables for PromptLearner.forward (coop.py:259-296).

    Returns (src_map [C,L] int32, ctx_pos [C,n_ctx] int32, L):
    src_map[c,t] >= 0 -> row of the class's token embedding (prefix/class/suffix),
    src_map[c,t] < 0  -> context vector (-1 - m).
    L = max(EOT)+1 when truncating: positions after the EOT never reach it under the
    causal mask (model.py:592-598), so truncation is exact."""
    L = int(max(eot)) + 1 if truncate else 77
    src = np.zeros((n_cls, L), np.int32)
    cpos = np.zeros((n_cls, max(n_ctx, 1)), np.int32)
    for c in range(n_cls):
        nl = int(name_lens[c]) if name_lens is not None else 0
        if position == "end":
            seq = [0] + [-1 - k for k in range(n_ctx)] + list(range(1 + n_ctx, 77))
        elif position == "middle":
            h = n_ctx // 2
            seq = ([0] + [-1 - k for k in range(h)] + [1 + n_ctx + j for j in range(nl)]
                   + [-1 - k for k in range(h, n_ctx)] + list(range(1 + n_ctx + nl, 77)))
        elif position == "front":
            seq = ([0] + [1 + n_ctx + j for j in range(nl)] + [-1 - k for k in range(n_ctx)]
                   + list(range(1 + n_ctx + nl, 77)))
        else:
            raise ValueError("Unknown class_token_position")
        assert len(seq) == 77
        src[c] = seq[:L]
        for t, m in enumerate(seq):
            if m < 0:
                if t >= L:
                    raise ValueError("context slot past the EOT token")
                cpos[c, -1 - m] = t
    return src, cpos, L


class PromptAssembleFn(torch.autograd.Function):
    """x0[(b*C+c)*L+t] = prompt token (+ctx[+bias_b]) + pos[t] (or the shared-prefix packed
    rows, PromptLayout.pack); grads to ctx (and bias)."""

    @staticmethod
    def forward(ctx, ctx_vec, bias, lay):
        B = 1 if bias is None else bias.shape[0]
        csc = ctx_vec.dim() == 3
        W = ctx_vec.shape[-1]
        sc = lay.n_ctx * W if csc else 0
        bias_c = None if bias is None else bias.contiguous()
        if lay.pack is not None:  # shared-prefix packed rows [B*R, W]
            x0 = ops.prompt_assemble_rows(B, lay.R, lay.n_cls, lay.L, lay.row_tab, lay.src_map, lay.emb,
                                          ctx_vec.contiguous(), 0, sc, bias_c, lay.pos)
        else:
            x0 = ops.prompt_assemble(B, lay.n_cls, lay.L, lay.src_map, lay.emb, ctx_vec.contiguous(), 0, sc,
                                     bias_c, lay.pos)
        ctx.lay, ctx.B, ctx.csc, ctx.shape, ctx.has_bias = lay, B, csc, ctx_vec.shape, bias is not None
        return x0

    @staticmethod
    def backward(ctx, dx0):
        lay = ctx.lay
        W = ctx.shape[-1]
        if lay.pack is not None:
            if not ctx.csc and (ctx.B > 1 or ctx.has_bias):
                # the per-image slot gradients summed into d ctx and d bias in the same launch (no
                # separate reductions; clipk_ctx_bias_grad_rows)
                dctx, dbias = ops.ctx_bias_grad_rows(ctx.B, lay.R, W, lay.n_ctx, lay.slot_ptr, lay.slot_rows,
                                                     dx0.contiguous(), bias=ctx.has_bias)
                return dctx.view(ctx.shape), dbias, None
            d = ops.ctx_grad_rows(ctx.B, lay.R, W, lay.n_ctx, lay.slot_ptr, lay.slot_rows, dx0.contiguous())
        else:
            d = ops.ctx_grad(ctx.B, lay.n_cls, lay.L, W, lay.n_ctx, ctx.csc, lay.ctx_pos, dx0.contiguous())
        if ctx.csc:
            return d.view(ctx.shape), None, None
        d = d.view(ctx.B, lay.n_ctx, W)
        dctx = d.sum(0) if ctx.B > 1 else d[0]
        dbias = d.sum(1) if ctx.has_bias else None
        return dctx, dbias, None


class CosineLogitsFn(torch.autograd.Function):
    """logits = scale * cos(imf[b], txt[row]); row = b*C+c (per_image) or c."""

    @staticmethod
    def forward(ctx, imf, txt, scale, per_image, n_cls):
        imf = imf.contiguous()
        txt = txt.contiguous()
        logits, inv_t, inv_i = ops.cosine_logits(imf, txt, scale, per_image, n_cls)
        ctx.save_for_backward(imf, txt, inv_t, inv_i)
        ctx.scale, ctx.per_image = scale, per_image
        return logits

    @staticmethod
    def backward(ctx, dlogits):
        imf, txt, inv_t, inv_i = ctx.saved_tensors
        dtxt = ops.cosine_logits_bwd(imf, txt, inv_t, inv_i, dlogits.contiguous(), ctx.scale, ctx.per_image)
        return None, dtxt, None, None, None


class CrossEntropyFn(torch.autograd.Function):
    """nn.CrossEntropyLoss (mean) or MultiClassFocalLoss (coop.py:145-163) with the reference's
    reductions 'mean' | 'sum' | 'none' (coop.py:158-163), fused fwd+bwd."""

    @staticmethod
    def forward(ctx, logits, labels, alpha, gamma, focal, reduction="mean"):
        B = logits.shape[0]
        ctx.reduction = reduction
        if reduction in ("mean", "sum") and B > 0:
            # the batch reduction in the loss launch itself (clipk_ce_loss_reduce)
            loss, ctx.dl = ops.ce_loss_reduce(logits.contiguous(), labels, alpha, gamma, focal,
                                              grad=logits.requires_grad, reduction=reduction)
            return loss
        scale = 1.0 / B if reduction == "mean" else 1.0
        row, dl = ops.ce_loss(logits.contiguous(), labels, alpha, gamma, focal, grad=logits.requires_grad,
                              grad_scale=scale)
        ctx.dl = dl
        if reduction == "mean":
            return row.mean()
        if reduction == "sum":
            return row.sum()
        return row

    @staticmethod
    def backward(ctx, g):
        # 'none': g is [B], each row's gradient scales its own row of d(row loss)/d logits. A
        # scalar loss back-propagated from backward_unit's cached 1.0 (every trainer step) needs
        # no multiply launch
        if ctx.reduction != "none" and g.data_ptr() == unit_grad(g.device).data_ptr():
            return ctx.dl, None, None, None, None, None
        dl = ctx.dl * (g[:, None] if ctx.reduction == "none" else g)
        return dl, None, None, None, None, None


_UNIT = {}


def unit_grad(device):
    """The cached scalar 1.0 a trainer step back-propagates from (backward_unit); read-only."""
    key = str(device)
    t = _UNIT.get(key)
    if t is None:
        t = _UNIT[key] = torch.ones((), device=device)
    return t


def backward_unit(loss):
    """loss.backward() from the cached unit gradient: no per-step fill launch for the seed, and
    CrossEntropyFn.backward skips its multiply by it (bitwise loss.backward())."""
    loss.backward(unit_grad(loss.device))


class MetaNetNormFn(torch.autograd.Function):
    """MetaNetFn on the L2-normalised rows of x (cocoop.py:238 imf / imf.norm(dim=-1) folded into
    the Meta-Net launch, clipk_meta_net_fwd_norm): returns (y, xn); xn (the normalised features,
    for the cosine logits) carries no gradient (the image encoder is frozen)."""

    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2):
        xn, h, y = ops.meta_net(x.contiguous(), w1.contiguous(), b1.contiguous(), w2.contiguous(), b2.contiguous(),
                                normalize=True)
        ctx.save_for_backward(xn, h, w2)
        ctx.dims = (x.shape[1], w1.shape[0], w2.shape[0])
        ctx.mark_non_differentiable(xn)
        ctx.set_materialize_grads(False)  # (no zero-filled gradient launched for xn)
        return y, xn

    @staticmethod
    def backward(ctx, dy, dxn):
        if dy is None:
            return None, None, None, None, None
        xn, h, w2 = ctx.saved_tensors
        V, Hd, Wd = ctx.dims
        dw1, db1, dw2, db2 = ops.meta_net_bwd(xn, h, w2.contiguous(), dy, V, Hd, Wd)
        return None, dw1, db1, dw2, db2


class MetaNetFn(torch.autograd.Function):
    """CoCoOp meta_net (cocoop.py:139-143): Linear(V,V/16) -> ReLU -> Linear(V/16,W)."""

    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2):
        x = x.contiguous()
        h, y = ops.meta_net(x, w1.contiguous(), b1.contiguous(), w2.contiguous(), b2.contiguous())
        ctx.save_for_backward(x, h, w2)
        ctx.dims = (x.shape[1], w1.shape[0], w2.shape[0])
        return y

    @staticmethod
    def backward(ctx, dy):
        x, h, w2 = ctx.saved_tensors
        V, Hd, Wd = ctx.dims
        dw1, db1, dw2, db2 = ops.meta_net_bwd(x, h, w2.contiguous(), dy, V, Hd, Wd)
        return None, dw1, db1, dw2, db2
