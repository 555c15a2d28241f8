"""CLIP on MI355X: packed frozen weights + native encoders behind autograd Functions.

Mirrors the pieces of ``PromptSRC/clip/model.py`` that the CoOp/CoCoOp trainers use
(``build_model`` 662-705; ``CLIP`` attributes ``visual``, ``token_embedding``,
``positional_embedding``, ``ln_final``, ``text_projection``, ``logit_scale``, ``dtype``),
but the encoders run as libclipk.so launch sequences:

* ``VisionEncoder``  — VisionTransformer.forward (model.py:401-431), frozen; with
  ``with_grad`` also the prompted ViT of IVLP / MaPLe / PromptSRC (visual prompt rows after the
  image tokens + deep prompts, model.py:191-331, 434-485) with its input-grad backward,
  exposed through ``PromptedVisionFn``.
* ``TextEncoderCore`` — the text Transformer + ln_final + text_projection
  (TextEncoder.forward, trainers/coop.py:195-205) with a native input-grad backward
  (weights frozen: coop.py:419-421), exposed through ``TextEncodeFn`` (``DeepTextEncodeFn``:
  with per-layer deep prompts).

Precision (cfg ``PREC``; PREC_DTYPES): "fp32" -> fp32 operands on f32-input MFMA, fp32
residual stream (parity mode); "fp32s" -> the fp32 mode's dataflow (fp32 activations, residual
stream, LayerNorm, attention) with every GEMM on the 16-bit MFMA as a split-fp16 product
(weights packed once by clipk_split_pack; include/clipk.h CLIPK_F32S): fp32-class results, the
north-star 1e-3 logit bar, at several times the f32-MFMA rate; "fp16" -> fp16 forward and backward GEMM operands, a 16-bit
text residual stream and residual-gradient stream; "amp" -> fp16 forward, bf16 backward
operands; "bf16" -> bf16 both. LayerNorm statistics, softmax and MFMA accumulation are fp32
in every mode. The reference's own "fp16" runs in fp32 (convert_weights disabled,
model.py:699), so the 16-bit modes are judged against the fp32 oracle.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np
import torch
import torch.nn as nn

from .. import _native as N
from .. import ops
from .synth import ClipArch

PREC_DTYPES = {
    "fp32": (torch.float32, torch.float32),
    "fp32s": (torch.float32, torch.float32),
    "fp16": (torch.float16, torch.float16),
    "amp": (torch.float16, torch.bfloat16),
    "bf16": (torch.bfloat16, torch.bfloat16),
}



def prec_dtypes(prec):
    """(activation dtype, text-backward gradient dtype) of a PREC. The reference's PREC fp16
    actually runs fp32 (convert_weights is disabled, PromptSRC/clip/model.py:699),
    so the build's 16-bit modes are judged against the fp32 oracle (tests/test_parity_gpu.py).
    PREC fp16 backpropagates in fp16: against the oracle its input gradients measure
    1-cos <= 5e-5, bf16 gradients 1.5e-3. CLIPK_GRAD_BF16=1 switches to bf16 (more range)."""
    import os
    act, grad = PREC_DTYPES[prec]
    if prec == "fp16" and os.environ.get("CLIPK_GRAD_BF16", "0") not in ("", "0"):
        grad = torch.bfloat16
    return act, grad


_LAYER_KEYS = ["ln_1.weight", "ln_1.bias", "attn.in_proj_weight", "attn.in_proj_bias",
               "attn.out_proj.weight", "attn.out_proj.bias", "ln_2.weight", "ln_2.bias",
               "mlp.c_fc.weight", "mlp.c_fc.bias", "mlp.c_proj.weight", "mlp.c_proj.bias"]


def _mm_weight(x, device, act, split):
    """A GEMM weight [N, K] as the encoder consumes it: in the activation dtype, or (PREC fp32s)
    split-packed for the split-fp16 GEMM (ops.split_pack)."""
    x = x.to(device, torch.float32 if split else act).contiguous()
    return ops.split_pack(x) if split else x


def split_mode(weights) -> int:
    """clipk_encoder_set_split mode of a PREC fp32s encoder: 2 when every split-packed GEMM weight
    it was created with is fp16-valued (ops.split_lo_zero; the released CLIP checkpoints are fp16,
    PromptSRC/clip/clip.py:154-180), so those GEMMs run CLIPK_F32S16 on the compact weights
    (compact16: 2 MFMAs per product, half of B's bytes, the same results); else 1. Knob
    FSP_SPLIT_W16=0 keeps 1 (A/B)."""
    if os.environ.get("FSP_SPLIT_W16", "1") == "0":
        return 1
    packed = [t for t in weights if isinstance(t, torch.Tensor) and t.dtype == torch.int32]
    return 2 if packed and all(ops.split_lo_zero(t) for t in packed) else 1


def compact16(tensors):
    """Split mode 2's weight tables: every split-packed (int32) weight replaced by its compact fp16
    form (ops.split_hi16, the CLIPK_F32S16 B operand); other entries unchanged."""
    return [ops.split_hi16(t) if isinstance(t, torch.Tensor) and t.dtype == torch.int32 else t for t in tensors]


def _t(v):
    return torch.as_tensor(np.asarray(v)) if not isinstance(v, torch.Tensor) else v.detach()


def arch_from_state_dict(sd) -> ClipArch:
    """Infer the ViT CLIP shape from state-dict shapes (model.py:663-687)."""
    if "visual.proj" not in sd:
        raise KeyError("only ViT CLIP backbones are on this path (ModifiedResNet is out of scope)")
    D = _t(sd["visual.conv1.weight"]).shape[0]
    layers = len([k for k in sd if k.startswith("visual.") and k.endswith(".attn.in_proj_weight")])
    p = _t(sd["visual.conv1.weight"]).shape[-1]
    grid = round((_t(sd["visual.positional_embedding"]).shape[0] - 1) ** 0.5)
    W = _t(sd["ln_final.weight"]).shape[0]
    tl = len({k.split(".")[2] for k in sd if k.startswith("transformer.resblocks")})
    return ClipArch(embed_dim=_t(sd["text_projection"]).shape[1], image_resolution=p * grid,
                    vision_layers=layers, vision_width=D, vision_patch_size=p,
                    context_length=_t(sd["positional_embedding"]).shape[0],
                    vocab_size=_t(sd["token_embedding.weight"]).shape[0], transformer_width=W,
                    transformer_heads=W // 64, transformer_layers=tl)


class _Workspace:
    """Grow-only scratch arena per (device, slot, stream): stream-ordered reuse, caller-owned
    memory. Per stream because an encoder may run on two streams at once (the image encoder
    on the side stream of trainers/_vision.py beside an inline run on the main stream): one
    shared buffer would be a race."""

    def __init__(self):
        self.buf = {}

    def get(self, nbytes: int, device, slot: str = "ws") -> torch.Tensor:
        dev = torch.device(device)
        sid = torch.cuda.current_stream(dev).cuda_stream if dev.type == "cuda" else 0
        key = (str(dev), slot, sid)
        b = self.buf.get(key)
        if b is None or b.numel() < nbytes:
            b = torch.empty(max(nbytes, 1 << 20), dtype=torch.uint8, device=device)
            self.buf[key] = b
        return b


WORKSPACE = _Workspace()


def _ptrs(tensors):
    arr = (ctypes.c_void_p * len(tensors))()
    for i, t in enumerate(tensors):
        arr[i] = None if t is None else t.data_ptr()
    return arr


def ln_fold_enabled() -> bool:
    """Knob FSP_LN_FOLD=0 builds 16-bit text encoders without the LayerNorm fold."""
    return os.environ.get("FSP_LN_FOLD", "1") != "0"


def ln_fold_weights(w, b, gamma, beta, act, device, split=False, gamma_on_a=False):
    """LayerNorm folded into the Linear that consumes it (include/clipk.h, clipk_gemm_ln):
    LN(x) W^T + b = rstd * (x W'^T - mean * s) + c with W' = W diag(gamma) in the operand dtype,
    s = W' summed over its input dimension (of the rounded W'), c = b + W beta.
    ``split`` (PREC fp32s): W' fp32, split-packed (ops.split_pack), and s summed over the value
    the split GEMM multiplies by, (hi + lo) / SPLIT_SCALE, so the mean term cancels against it.
    ``gamma_on_a`` (split mode 2, clipk_gemm_ln_gamma): B = W itself in its compact fp16 form
    (ops.split_hi16), gamma applied to A in the kernel; s = rowsums of W diag(gamma) over W's
    packed value.
    Returns (W', s, c) on ``device``, or None when W' does not fit the operand dtype."""
    wd = w.double()
    if gamma_on_a:
        x = w.float() * N.SPLIT_SCALE
        hi = x.half().float()
        lo = (x - hi).half().float()
        s = (((hi.double() + lo.double()) / N.SPLIT_SCALE) * gamma.double()[None, :]).sum(1).float()
        c = (b.double() + wd @ beta.double()).float()
        wdev = ops.split_hi16(ops.split_pack(w.float().to(device).contiguous()))
        return (wdev, s.to(device).contiguous(), c.to(device).contiguous())
    wp = (wd * gamma.double()[None, :]).to(act)
    if not bool(torch.isfinite(wp.float()).all()):
        return None
    if split:
        x = wp.float() * N.SPLIT_SCALE
        if not float(x.abs().max()) < 65504.0:
            return None
        hi = x.half().float()
        lo = (x - hi).half().float()  # x - hi is exact in fp32, as in clipk_split_pack
        s = ((hi.double() + lo.double()) / N.SPLIT_SCALE).sum(1).float()
        wdev = ops.split_pack(wp.float().to(device).contiguous())
    else:
        s = wp.double().sum(1).float()
        wdev = wp.to(device).contiguous()
    c = (b.double() + wd @ beta.double()).float()
    return (wdev, s.to(device).contiguous(), c.to(device).contiguous())


class SplitStatus:
    """The overflow flags of a device's PREC fp32s encoders (clipk_encoder_set_status): one device
    int the text and image encoders OR into -- 1: a forward's features came out non-finite, 2: a
    backward's gradients did. A backward reads them at once (its overflow re-runs at a lower scale,
    TextEncoderCore.backward); inference forwards do not synchronise for them: they are read every
    READ_EVERY forward-only calls and by check() (TrainerX.test calls it after its last batch), so a
    non-finite forward still raises, within that many calls, without a host stall per batch."""
    READ_EVERY = 64
    _by_device = {}

    def __init__(self, device):
        self.flags = torch.zeros(1, dtype=torch.int32, device=device)
        # the host-visible word clipk_status_take hands the flags to (pinned: the kernel writes it,
        # no runtime copy or fill launch per read)
        self.host = torch.zeros(1, dtype=torch.int32, pin_memory=True)
        self.pending = 0  # forward-only calls since the last read

    @classmethod
    def of(cls, device):
        key = str(torch.device(device))
        if key not in cls._by_device:
            cls._by_device[key] = cls(device)
        return cls._by_device[key]

    def read(self):
        """Read and clear the flags (one synchronisation); a non-finite forward raises. Returns
        the backward flag."""
        ops.status_take(self.flags, self.host)  # host <- flags, flags <- 0 (one clipk launch)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.flags.device))
        ev.synchronize()
        st = int(self.host[0])
        self.pending = 0
        if st & 1:
            raise N.ClipkError("PREC fp32s encoder: non-finite features -- an activation exceeded fp16's range "
                               "(65504) in the split-fp16 GEMM operands; use PREC fp32")
        return bool(st & 2)

    def take_async(self):
        """Hand the flags to a pinned word and clear them at this point of the current stream,
        without waiting: returns a handle whose result() waits for that point only (a ring of
        two words: the previous step's handle stays valid while the next one is taken)."""
        ring = getattr(self, "_ring", None)
        if ring is None:
            ring = self._ring = [torch.zeros(1, dtype=torch.int32, pin_memory=True) for _ in range(2)]
            self._ri = 0
        host = ring[self._ri]
        self._ri ^= 1
        ops.status_take(self.flags, host)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.flags.device))
        return _StatusHandle(ev, host)

    def forward_done(self):
        self.pending += 1
        if self.pending >= self.READ_EVERY:
            self.read()

    def check(self):
        """The deferred read of the inference forwards' flags."""
        if self.pending:
            self.read()


class _StatusHandle:
    """SplitStatus.take_async's result: the flags as of that stream point (a non-finite forward
    raises, as SplitStatus.read)."""

    def __init__(self, ev, host):
        self.ev, self.host = ev, host

    def result(self):
        self.ev.synchronize()
        st = int(self.host[0])
        if st & 1:
            raise N.ClipkError("PREC fp32s encoder: non-finite features -- an activation exceeded fp16's range "
                               "(65504) in the split-fp16 GEMM operands; use PREC fp32")
        return st


def check_split_status(device=None):
    """SplitStatus.check() for every device with PREC fp32s encoders (or the given one)."""
    for key, st in list(SplitStatus._by_device.items()):
        if device is None or key == str(torch.device(device)):
            st.check()


class _Encoder:
    handle = None

    def __del__(self):
        if self.handle is not None:
            try:
                N.load().clipk_encoder_destroy(self.handle)
            except Exception:
                pass
            self.handle = None


class TextEncoderCore(_Encoder):
    """Packed text transformer + ln_final + projection; native fwd / input-grad bwd."""

    def __init__(self, sd, arch: ClipArch, prec: str, device, with_grad: bool = True):
        act, grad = prec_dtypes(prec)
        self.arch, self.prec, self.device = arch, prec, torch.device(device)
        self.act, self.grad = act, grad
        split = prec == "fp32s"
        W, nl = arch.transformer_width, arch.transformer_layers
        self.W, self.E, self.layers, self.heads = W, arch.embed_dim, nl, W // 64
        keep = []
        table = []
        # LayerNorm fold of ln_1 / ln_2 into in_proj / c_fc (16-bit encoders and PREC fp32s;
        # clipk_encoder_set_ln_fold)
        fold = [] if (act != torch.float32 or split) and ln_fold_enabled() else None
        params = []
        for i in range(nl):
            p = {k: _t(sd[f"transformer.resblocks.{i}.{k}"]).float() for k in _LAYER_KEYS}
            params.append(p)
            f32 = lambda x: x.to(self.device, torch.float32).contiguous()
            A = lambda x: _mm_weight(x, self.device, act, split)
            G = lambda x: _mm_weight(x.t(), self.device, grad, split) if with_grad else None
            row = [f32(p["ln_1.weight"]), f32(p["ln_1.bias"]), A(p["attn.in_proj_weight"]),
                   f32(p["attn.in_proj_bias"]), A(p["attn.out_proj.weight"]), f32(p["attn.out_proj.bias"]),
                   f32(p["ln_2.weight"]), f32(p["ln_2.bias"]), A(p["mlp.c_fc.weight"]), f32(p["mlp.c_fc.bias"]),
                   A(p["mlp.c_proj.weight"]), f32(p["mlp.c_proj.bias"]),
                   G(p["attn.in_proj_weight"]), G(p["attn.out_proj.weight"]), G(p["mlp.c_fc.weight"]),
                   G(p["mlp.c_proj.weight"])]
            keep += row
            table += row
        P = _t(sd["text_projection"]).float()
        head = [_t(sd["ln_final.weight"]).float().to(self.device).contiguous(),
                _t(sd["ln_final.bias"]).float().to(self.device).contiguous(),
                _mm_weight(P.t(), self.device, act, split),
                _mm_weight(P, self.device, grad, split) if with_grad else None]
        keep += head
        self._keep = keep
        # PREC fp32s split mode (2: fp16-valued weights, CLIPK_F32S16), decided before the fold:
        # mode 2 folds gamma into A (clipk_gemm_ln_gamma) so B stays the fp16-valued W
        self.split_mode = split_mode(keep) if split else 0
        if self.split_mode == 2:  # the tables hold the compact weights (clipk_encoder_set_split)
            table, head = compact16(table), compact16(head)
            keep = table + head
            self._keep = keep
        for p in params:
            if fold is None:
                break
            ga = self.split_mode == 2
            f_in = ln_fold_weights(p["attn.in_proj_weight"], p["attn.in_proj_bias"], p["ln_1.weight"],
                                   p["ln_1.bias"], act, self.device, split, gamma_on_a=ga)
            f_fc = ln_fold_weights(p["mlp.c_fc.weight"], p["mlp.c_fc.bias"], p["ln_2.weight"],
                                   p["ln_2.bias"], act, self.device, split, gamma_on_a=ga)
            fold = fold + list(f_in) + list(f_fc) if f_in and f_fc else None
        h = ctypes.c_void_p()
        N.check(N.load().clipk_encoder_create(W, nl, self.heads, self.E, ops.DT[act], ops.DT[grad],
                                              _ptrs(table), _ptrs(head), ctypes.byref(h)),
                "clipk_encoder_create(text)")
        self.handle = h
        self._status = None
        if split:
            N.check(N.load().clipk_encoder_set_split(h, self.split_mode), "clipk_encoder_set_split(text)")
            # overflow flags of the split calls (clipk_encoder_set_status; SplitStatus): 1 = a
            # forward's features, 2 = a backward's gradients came out non-finite
            self._status = SplitStatus.of(self.device)
            N.check(N.load().clipk_encoder_set_status(h, ops._p(self._status.flags)), "clipk_encoder_set_status")
            N.check(N.load().clipk_encoder_set_split_target(h, self.SPLIT_TARGET), "clipk_encoder_set_split_target")
        if fold:
            self._keep += fold
            N.check(N.load().clipk_encoder_set_ln_fold(h, _ptrs(fold)), "clipk_encoder_set_ln_fold")

    def set_deep(self, deep, rows, n_per, grads=None):
        """Deep prompts for the next call(s): deep fp32 [n_deep, n_ctx, W] (None clears)."""
        if deep is None:
            N.check(N.load().clipk_encoder_set_deep_prompts(self.handle, 0, 0, 0, None, None, None),
                    "clipk_encoder_set_deep_prompts")
            return
        N.check(N.load().clipk_encoder_set_deep_prompts(self.handle, deep.shape[0], deep.shape[1], n_per, ops._p(rows),
                                                        ops._p(deep), ops._p(grads)),
                "clipk_encoder_set_deep_prompts")

    def _input_rows(self, lib, shape):
        """clipk_encoder_set_input_rows for this call: 1 when the packed layout's class rows are
        the same in every group and only its prefix rows need an input gradient
        (TextShape.prefix_input); forward and backward of one call see the same mode."""
        N.check(lib.clipk_encoder_set_input_rows(self.handle, int(bool(getattr(shape, "prefix_input", False)))),
                "clipk_encoder_set_input_rows")

    def forward(self, x0, shape, save):
        """x0 fp32 [shape.rows, W] -> txt fp32 [shape.nout, E] (+ saved arena if save)."""
        lib = N.load()
        h = self.handle
        txt = torch.empty(shape.nout, self.E, device=x0.device, dtype=torch.float32)
        if shape.packed:
            dims = (shape.G, shape.C, shape.R)
            wsb = lib.clipk_text_packed_ws_bytes(h, *dims)
            sb = lib.clipk_text_packed_saved_bytes(h, *dims) if save else 0
        else:
            wsb = lib.clipk_text_ws_bytes(h, shape.nseq, shape.L)
            sb = lib.clipk_text_saved_bytes(h, shape.nseq, shape.L) if save else 0
        ws = WORKSPACE.get(wsb, x0.device, "text_fwd")
        saved = torch.empty(sb, dtype=torch.uint8, device=x0.device) if save else None
        tail = (ops._p(x0), ops._p(shape.eot_rows), ops._p(txt), ops._p(saved), sb, ops._p(ws), ws.numel(),
                ops._stream())
        self._input_rows(lib, shape)
        if shape.packed:
            N.check(lib.clipk_text_forward_packed(h, shape.G, shape.C, shape.P, shape.R, shape.ntiles,
                                                  ops._p(shape.tiles), ops._p(shape.row_first), *tail),
                    "clipk_text_forward_packed")
        else:
            N.check(lib.clipk_text_forward(h, shape.nseq, shape.L, *tail), "clipk_text_forward")
        if self._status is not None and not save:
            self._status.forward_done()  # inference: read every READ_EVERY calls / SplitStatus.check
        return txt, saved

    # PREC fp32s: an overflowed backward is re-run once with this much lower scale target (10 more
    # bits of headroom below fp16's 65504 for gradient growth through the layers)
    SPLIT_TARGET, SPLIT_RETRY_TARGET = 7, -3

    def _check_status(self):
        """Read and clear the split overflow flags (one host synchronisation); a non-finite
        forward raises. Returns the backward flag."""
        return self._status.read()

    def backward(self, dtxt, shape, saved):
        lib = N.load()
        h = self.handle
        dx0 = torch.empty(shape.rows, self.W, device=dtxt.device, dtype=torch.float32)
        if shape.packed:
            wsb = lib.clipk_text_packed_bwd_ws_bytes(h, shape.G, shape.C, shape.R, shape.ntiles)
        else:
            wsb = lib.clipk_text_bwd_ws_bytes(h, shape.nseq, shape.L)
        ws = WORKSPACE.get(wsb, dtxt.device, "text_bwd")
        tail = (ops._p(shape.eot_rows), ops._p(dtxt.contiguous()), ops._p(saved), saved.numel(), ops._p(dx0),
                ops._p(ws), ws.numel(), ops._stream())
        self._input_rows(lib, shape)

        def run():
            if shape.packed:
                N.check(lib.clipk_text_backward_packed(h, shape.G, shape.C, shape.P, shape.R, shape.ntiles,
                                                       ops._p(shape.tiles), ops._p(shape.row_first), *tail),
                        "clipk_text_backward_packed")
            else:
                N.check(lib.clipk_text_backward(h, shape.nseq, shape.L, *tail), "clipk_text_backward")

        run()
        # (defer_check: the trainer reads the flag later, its SGD launch guarded by it on the
        # device -- CoCoOp._settle_pending re-runs an overflowed step with this check on)
        if self._status is not None and not self.defer_check and self._check_status():
            # the gradients overflowed the split operands' fp16 range: once more at a lower scale
            # target (exact: the backward is linear in dtxt and the scale a power of two)
            type(self).split_retries += 1
            N.check(lib.clipk_encoder_set_split_target(h, self.SPLIT_RETRY_TARGET), "clipk_encoder_set_split_target")
            try:
                run()
            finally:
                lib.clipk_encoder_set_split_target(h, self.SPLIT_TARGET)
            if self._check_status():
                raise N.ClipkError("PREC fp32s text encoder backward: non-finite gradients even at the lowered "
                                   "scale target (gradient growth beyond fp16's range); use PREC fp32")
        return dx0

    split_retries = 0  # PREC fp32s backwards re-run at the lower scale target (overflow), all instances
    defer_check = False


class TextEncodeFn(torch.autograd.Function):
    """x0 fp32 [shape.rows, W] (prompts + positional embedding) -> text features
    [shape.nout, E]; ``shape`` is a trainers.prompt_base.TextShape (plain or packed)."""

    @staticmethod
    def forward(ctx, x0, core, shape):
        txt, saved = core.forward(x0.contiguous(), shape, save=bool(ctx.needs_input_grad[0]))
        ctx.core, ctx.shape, ctx.saved_arena = core, shape, saved
        return txt

    @staticmethod
    def backward(ctx, dtxt):
        if ctx.saved_arena is None:
            raise RuntimeError("text encoder backward without saved activations")
        dx0 = ctx.core.backward(dtxt, ctx.shape, ctx.saved_arena)
        ctx.saved_arena = None
        return dx0, None, None


def deep_text_rows(shape, n_ctx, device):
    """Rows the text deep prompts replace (tokens 1..n_ctx of every sequence, model.py:244-252),
    as the [n_ctx][n_per] table of clipk_rows_inject: packed layout -> prefix rows of each group."""
    if shape.packed:
        base, n_per, stride = 1, shape.G, shape.R
    else:
        base, n_per, stride = 1, shape.nseq, shape.L
    p = torch.arange(n_ctx, dtype=torch.int64)[:, None]
    i = torch.arange(n_per, dtype=torch.int64)[None, :]
    return (i * stride + base + p).reshape(-1).to(torch.int32).to(device), n_per


class DeepTextEncodeFn(torch.autograd.Function):
    """TextEncodeFn with deep prompts (IVLP / MaPLe / PromptSRC text side, model.py:229-256 /
    287-331): deep fp32 [n_deep, n_ctx, W] replace rows 1..n_ctx before layers 1..n_deep."""

    @staticmethod
    def forward(ctx, x0, deep, core, shape):
        rows, n_per = deep_text_rows(shape, deep.shape[1], x0.device)
        deep = deep.contiguous()
        core.set_deep(deep, rows, n_per)
        try:
            txt, saved = core.forward(x0.contiguous(), shape, save=any(ctx.needs_input_grad[:2]))
        finally:
            core.set_deep(None, None, 0)
        ctx.core, ctx.shape, ctx.saved_arena = core, shape, saved
        ctx.deep, ctx.rows, ctx.n_per = deep, rows, n_per
        return txt

    @staticmethod
    def backward(ctx, dtxt):
        if ctx.saved_arena is None:
            raise RuntimeError("text encoder backward without saved activations")
        ddeep = torch.empty_like(ctx.deep)
        ctx.core.set_deep(ctx.deep, ctx.rows, ctx.n_per, ddeep)
        try:
            dx0 = ctx.core.backward(dtxt, ctx.shape, ctx.saved_arena)
        finally:
            ctx.core.set_deep(None, None, 0)
        ctx.saved_arena = None
        return dx0, ddeep, None, None


class VisionEncoder(nn.Module, _Encoder):
    """ViT image encoder on the native path: image [B,3,R,R] fp32 -> [B,E] fp32. Frozen
    weights; ``with_grad`` packs the transposed layer weights for the prompted input-grad
    backward (forward_prompted / PromptedVisionFn)."""

    def __init__(self, sd, arch: ClipArch, prec: str, device, with_grad: bool = False):
        nn.Module.__init__(self)
        act, _ = PREC_DTYPES[prec]
        split = prec == "fp32s"
        self.arch, self.act, self.dev = arch, act, torch.device(device)
        self.input_resolution = arch.image_resolution
        self.output_dim = arch.embed_dim
        D, nl, p = arch.vision_width, arch.vision_layers, arch.vision_patch_size
        f32 = lambda x: _t(x).float().to(self.dev).contiguous()
        A = lambda x: _mm_weight(_t(x).float(), self.dev, act, split)
        G = lambda x: _mm_weight(_t(x).float().t(), self.dev, act, split) if with_grad else None
        self.with_grad = with_grad
        table = []
        # LayerNorm fold of ln_1 / ln_2 for the layer-loop forward (clipk_vit_forward: 16-bit
        # residual stream, or PREC fp32s's fp32 one), built once the split mode is known
        fparams = [] if (act != torch.float32 or split) and ln_fold_enabled() else None
        for i in range(nl):
            pre = f"visual.transformer.resblocks.{i}."
            q = {k: sd[pre + k] for k in _LAYER_KEYS}
            if fparams is not None:
                fparams.append({k: _t(v).float() for k, v in q.items()})
            table += [f32(q["ln_1.weight"]), f32(q["ln_1.bias"]), A(q["attn.in_proj_weight"]),
                      f32(q["attn.in_proj_bias"]), A(q["attn.out_proj.weight"]), f32(q["attn.out_proj.bias"]),
                      f32(q["ln_2.weight"]), f32(q["ln_2.bias"]), A(q["mlp.c_fc.weight"]), f32(q["mlp.c_fc.bias"]),
                      A(q["mlp.c_proj.weight"]), f32(q["mlp.c_proj.bias"]),
                      G(q["attn.in_proj_weight"]), G(q["attn.out_proj.weight"]), G(q["mlp.c_fc.weight"]),
                      G(q["mlp.c_proj.weight"])]
        k = 3 * p * p
        kq = 32 if act == torch.float32 else 64
        self.Kp = (k + kq - 1) // kq * kq
        conv = torch.zeros(D, self.Kp)
        conv[:, :k] = _t(sd["visual.conv1.weight"]).float().reshape(D, k)
        head = [f32(sd["visual.ln_pre.weight"]), f32(sd["visual.ln_pre.bias"]),
                f32(sd["visual.ln_post.weight"]), f32(sd["visual.ln_post.bias"]),
                _mm_weight(_t(sd["visual.proj"]).float().t(), self.dev, act, split),
                _mm_weight(conv, self.dev, act, split), f32(sd["visual.class_embedding"]),
                f32(sd["visual.positional_embedding"])]
        # backward of the head: d ln_post(CLS) = dfeat . proj^T  (proj [D, E], B operand [N=D, K=E])
        self.proj_bwd = _mm_weight(_t(sd["visual.proj"]).float(), self.dev, act, split) if with_grad else None
        self.split_mode = split_mode([t for t in table if t is not None] + head + [self.proj_bwd]) if split else 0
        if self.split_mode == 2:  # the tables hold the compact weights (clipk_encoder_set_split)
            table, head = compact16(table), compact16(head)
            self.proj_bwd = compact16([self.proj_bwd])[0]
        self._keep = [t for t in table if t is not None] + head
        fold = None
        if fparams is not None:
            ga = self.split_mode == 2  # mode 2: gamma on A, B = W itself (clipk_gemm_ln_gamma)
            fold = []
            for qf in fparams:
                f_in = ln_fold_weights(qf["attn.in_proj_weight"], qf["attn.in_proj_bias"], qf["ln_1.weight"],
                                       qf["ln_1.bias"], act, self.dev, split, gamma_on_a=ga)
                f_fc = ln_fold_weights(qf["mlp.c_fc.weight"], qf["mlp.c_fc.bias"], qf["ln_2.weight"],
                                       qf["ln_2.bias"], act, self.dev, split, gamma_on_a=ga)
                if not (f_in and f_fc):
                    fold = None
                    break
                fold += list(f_in) + list(f_fc)
        self.width, self.n_tokens = D, (arch.image_resolution // p) ** 2 + 1
        h = ctypes.c_void_p()
        N.check(N.load().clipk_vision_create(D, nl, D // 64, arch.embed_dim, arch.image_resolution, p,
                                             ops.DT[act], _ptrs(table), _ptrs(head), ctypes.byref(h)),
                "clipk_vision_create")
        self.handle = h
        self._status = None
        if split:
            N.check(N.load().clipk_encoder_set_split(h, self.split_mode), "clipk_encoder_set_split(vision)")
            # non-finite ViT features set flag 1 of the device's split status (the ViT's
            # split_check had no status to report to)
            self._status = SplitStatus.of(self.dev)
            N.check(N.load().clipk_encoder_set_status(h, ops._p(self._status.flags)), "clipk_encoder_set_status")
        if fold:
            self._keep += fold
            N.check(N.load().clipk_encoder_set_ln_fold(h, _ptrs(fold)), "clipk_encoder_set_ln_fold")

    def _check_image(self, image):
        image = image.to(self.dev, torch.float32).contiguous()
        if image.shape[1:] != (3, self.input_resolution, self.input_resolution):
            raise RuntimeError(f"expected [B,3,{self.input_resolution},{self.input_resolution}] images, "
                               f"got {tuple(image.shape)}")
        return image

    def deep_rows(self, B, n_vpt):
        """Rows the deep visual prompts replace: the last n_vpt rows of every image
        (model.py:234-241), as the [n_vpt][B] table of clipk_rows_inject."""
        Lp = self.n_tokens + n_vpt
        p = torch.arange(n_vpt, dtype=torch.int64)[:, None]
        b = torch.arange(B, dtype=torch.int64)[None, :]
        return (b * Lp + self.n_tokens + p).reshape(-1).to(torch.int32).to(self.dev)

    def set_deep(self, deep, rows, n_per, grads=None):
        lib = N.load()
        if deep is None or deep.shape[0] == 0:
            N.check(lib.clipk_encoder_set_deep_prompts(self.handle, 0, 0, 0, None, None, None),
                    "clipk_encoder_set_deep_prompts")
            return
        N.check(lib.clipk_encoder_set_deep_prompts(self.handle, deep.shape[0], deep.shape[1], n_per, ops._p(rows),
                                                   ops._p(deep), ops._p(grads)), "clipk_encoder_set_deep_prompts")

    def forward_prompted(self, image, vpt, deep=None, save=False):
        """image [B,3,R,R], vpt fp32 [n_vpt, D] (n_vpt may be 0), deep fp32 [n_deep, n_vpt, D]
        -> (feat [B, E] fp32, saved arena or None)."""
        image = self._check_image(image)
        B, n_vpt = image.shape[0], vpt.shape[0]
        lib = N.load()
        feat = torch.empty(B, self.output_dim, device=self.dev)
        wsb = lib.clipk_vit_prompted_ws_bytes(self.handle, B, n_vpt)
        ws = WORKSPACE.get(wsb, self.dev, "vitp")
        sb = lib.clipk_vit_prompted_saved_bytes(self.handle, B, n_vpt) if save else 0
        saved = torch.empty(sb, dtype=torch.uint8, device=self.dev) if save else None
        rows = self.deep_rows(B, n_vpt) if deep is not None and deep.shape[0] else None
        self.set_deep(deep, rows, B)
        try:
            N.check(lib.clipk_vit_forward_prompted(self.handle, B, ops._p(image), n_vpt, ops._p(vpt), ops._p(feat),
                                                   ops._p(saved), sb, ops._p(ws), ws.numel(), ops._stream()),
                    "clipk_vit_forward_prompted")
        finally:
            self.set_deep(None, None, 0)
        return feat, saved

    def backward_prompted(self, dfeat, vpt, deep, saved, B):
        """-> (d vpt [n_vpt, D], d deep [n_deep, n_vpt, D] or None)."""
        if not self.with_grad:
            raise RuntimeError("the image encoder was built without backward weights (with_grad=False)")
        lib = N.load()
        n_vpt = vpt.shape[0]
        dvpt = torch.empty_like(vpt)
        ddeep = torch.empty_like(deep) if deep is not None and deep.shape[0] else None
        wsb = lib.clipk_vit_prompted_ws_bytes(self.handle, B, n_vpt)
        ws = WORKSPACE.get(wsb, self.dev, "vitp")
        rows = self.deep_rows(B, n_vpt) if ddeep is not None else None
        self.set_deep(deep if ddeep is not None else None, rows, B, ddeep)
        try:
            N.check(lib.clipk_vit_backward_prompted(self.handle, B, n_vpt, ops._p(vpt), ops._p(self.proj_bwd),
                                                    ops._p(dfeat.contiguous()), ops._p(saved), saved.numel(),
                                                    ops._p(dvpt), ops._p(ws), ws.numel(), ops._stream()),
                    "clipk_vit_backward_prompted")
        finally:
            self.set_deep(None, None, 0)
        return dvpt, ddeep

    def forward(self, image):
        if image.requires_grad:
            raise RuntimeError("the image encoder is frozen and forward-only (no input grad)")
        image = self._check_image(image)
        B = image.shape[0]
        lib = N.load()
        feat = torch.empty(B, self.output_dim, device=self.dev)
        wsb = lib.clipk_vit_ws_bytes(self.handle, B)
        ws = WORKSPACE.get(wsb, self.dev, "vit")
        N.check(lib.clipk_vit_forward(self.handle, B, ops._p(image), ops._p(feat), ops._p(ws), ws.numel(),
                                      ops._stream()), "clipk_vit_forward")
        return feat

    def __del__(self):
        _Encoder.__del__(self)


class PromptedVisionFn(torch.autograd.Function):
    """(vpt [n_vpt, D], deep [n_deep, n_vpt, D], image) -> image features [B, E] through the
    prompted ViT; gradients flow to the prompts only (the image and the weights are frozen)."""

    @staticmethod
    def forward(ctx, vpt, deep, image, enc):
        vpt = vpt.contiguous()
        deep = deep.contiguous() if deep is not None else None
        need = ctx.needs_input_grad[0] or (deep is not None and ctx.needs_input_grad[1])
        feat, saved = enc.forward_prompted(image, vpt, deep, save=need)
        ctx.enc, ctx.saved_arena, ctx.B = enc, saved, image.shape[0]
        ctx.vpt, ctx.deep = vpt, deep
        return feat

    @staticmethod
    def backward(ctx, dfeat):
        if ctx.saved_arena is None:
            raise RuntimeError("image encoder backward without saved activations")
        dvpt, ddeep = ctx.enc.backward_prompted(dfeat, ctx.vpt, ctx.deep, ctx.saved_arena, ctx.B)
        ctx.saved_arena = None
        return dvpt, ddeep, None, None


class CLIP(nn.Module):
    """Container with the attributes the prompt learners read (model.py:488-561)."""

    def __init__(self, sd, prec: str = "fp16", device="cuda", text_grad: bool = True, vision_grad: bool = False):
        super().__init__()
        if prec not in PREC_DTYPES:
            raise AssertionError(f"PREC must be one of {list(PREC_DTYPES)}")
        arch = arch_from_state_dict(sd)
        self.arch, self.prec = arch, prec
        dev = torch.device(device)
        self.visual = VisionEncoder(sd, arch, prec, dev, with_grad=vision_grad)
        self.text = TextEncoderCore(sd, arch, prec, dev, with_grad=text_grad)
        W = arch.transformer_width
        self.token_embedding = nn.Embedding(arch.vocab_size, W)
        with torch.no_grad():
            self.token_embedding.weight.copy_(_t(sd["token_embedding.weight"]).float())
        self.token_embedding.requires_grad_(False)  # host-side, init-time lookups only
        self.positional_embedding = nn.Parameter(_t(sd["positional_embedding"]).float().to(dev),
                                                 requires_grad=False)
        self.ln_final_weight = _t(sd["ln_final.weight"]).float()
        self.logit_scale = nn.Parameter(_t(sd["logit_scale"]).float().reshape(()).to(dev), requires_grad=False)
        self.logit_scale_value = float(np.exp(float(_t(sd["logit_scale"]))))
        self.context_length = arch.context_length

    @property
    def dtype(self):
        return torch.float32  # host-facing tensors are fp32; kernels pick operand types


def build_model(state_dict, prec: str = "fp16", device="cuda", text_grad: bool = True,
                vision_grad: bool = False) -> CLIP:
    """build_model(state_dict) analogue (model.py:662-705) for the native path; vision_grad
    packs the ViT's backward weights (trainers whose visual prompts train)."""
    return CLIP(state_dict, prec=prec, device=device, text_grad=text_grad, vision_grad=vision_grad)
