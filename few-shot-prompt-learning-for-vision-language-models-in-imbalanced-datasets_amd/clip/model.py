"""CLIP on MI355X: packed frozen weights + native encoders behind autograd Functions.

Mirrors the pieces of ``PromptSRC/clip/model.py`` that the CoOp/CoCoOp trainers use
(``build_model`` 662-705; ``CLIP`` attributes ``visual``, ``token_embedding``,
``positional_embedding``, ``ln_final``, ``text_projection``, ``logit_scale``, ``dtype``),
but the encoders run as libclipk.so launch sequences:

* ``VisionEncoder``  — VisionTransformer.forward (model.py:401-431), frozen, forward only.
* ``TextEncoderCore`` — the text Transformer + ln_final + text_projection
  (TextEncoder.forward, trainers/coop.py:195-205) with a native input-grad backward
  (weights frozen: coop.py:419-421), exposed through ``TextEncodeFn``.

Precision (cfg ``PREC``; PREC_DTYPES): "fp32" -> fp32 operands on f32-input MFMA, fp32
residual stream (parity mode); "fp16" -> fp16 forward and backward GEMM operands, a 16-bit
text residual stream and residual-gradient stream; "amp" -> fp16 forward, bf16 backward
operands; "bf16" -> bf16 both. LayerNorm statistics, softmax and MFMA accumulation are fp32
in every mode. The reference's own "fp16" runs in fp32 (convert_weights disabled,
model.py:699), so the 16-bit modes are judged against the fp32 oracle.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch
import torch.nn as nn

from .. import _native as N
from .. import ops
from .synth import ClipArch

PREC_DTYPES = {
    "fp32": (torch.float32, torch.float32),
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
    """Grow-only per-device scratch arena (stream-ordered reuse, caller-owned memory)."""

    def __init__(self):
        self.buf = {}

    def get(self, nbytes: int, device, slot: str = "ws") -> torch.Tensor:
        key = (str(device), slot)
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
        W, nl = arch.transformer_width, arch.transformer_layers
        self.W, self.E, self.layers, self.heads = W, arch.embed_dim, nl, W // 64
        keep = []
        table = []
        for i in range(nl):
            p = {k: _t(sd[f"transformer.resblocks.{i}.{k}"]).float() for k in _LAYER_KEYS}
            f32 = lambda x: x.to(self.device, torch.float32).contiguous()
            A = lambda x: x.to(self.device, act).contiguous()
            G = lambda x: x.t().contiguous().to(self.device, grad) if with_grad else None
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
                P.t().contiguous().to(self.device, act),
                P.contiguous().to(self.device, grad) if with_grad else None]
        keep += head
        self._keep = keep
        h = ctypes.c_void_p()
        N.check(N.load().clipk_encoder_create(W, nl, self.heads, self.E, ops.DT[act], ops.DT[grad],
                                              _ptrs(table), _ptrs(head), ctypes.byref(h)),
                "clipk_encoder_create(text)")
        self.handle = h

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
        if shape.packed:
            N.check(lib.clipk_text_forward_packed(h, shape.G, shape.C, shape.P, shape.R, shape.ntiles,
                                                  ops._p(shape.tiles), ops._p(shape.row_first), *tail),
                    "clipk_text_forward_packed")
        else:
            N.check(lib.clipk_text_forward(h, shape.nseq, shape.L, *tail), "clipk_text_forward")
        return txt, saved

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
        if shape.packed:
            N.check(lib.clipk_text_backward_packed(h, shape.G, shape.C, shape.P, shape.R, shape.ntiles,
                                                   ops._p(shape.tiles), ops._p(shape.row_first), *tail),
                    "clipk_text_backward_packed")
        else:
            N.check(lib.clipk_text_backward(h, shape.nseq, shape.L, *tail), "clipk_text_backward")
        return dx0


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


class VisionEncoder(nn.Module, _Encoder):
    """Frozen ViT image encoder on the native path: image [B,3,R,R] fp32 -> [B,E] fp32."""

    def __init__(self, sd, arch: ClipArch, prec: str, device):
        nn.Module.__init__(self)
        act, _ = PREC_DTYPES[prec]
        self.arch, self.act, self.dev = arch, act, torch.device(device)
        self.input_resolution = arch.image_resolution
        self.output_dim = arch.embed_dim
        D, nl, p = arch.vision_width, arch.vision_layers, arch.vision_patch_size
        f32 = lambda x: _t(x).float().to(self.dev).contiguous()
        A = lambda x: _t(x).float().to(self.dev, act).contiguous()
        table = []
        for i in range(nl):
            pre = f"visual.transformer.resblocks.{i}."
            q = {k: sd[pre + k] for k in _LAYER_KEYS}
            table += [f32(q["ln_1.weight"]), f32(q["ln_1.bias"]), A(q["attn.in_proj_weight"]),
                      f32(q["attn.in_proj_bias"]), A(q["attn.out_proj.weight"]), f32(q["attn.out_proj.bias"]),
                      f32(q["ln_2.weight"]), f32(q["ln_2.bias"]), A(q["mlp.c_fc.weight"]), f32(q["mlp.c_fc.bias"]),
                      A(q["mlp.c_proj.weight"]), f32(q["mlp.c_proj.bias"]), None, None, None, None]
        k = 3 * p * p
        kq = 32 if act == torch.float32 else 64
        self.Kp = (k + kq - 1) // kq * kq
        conv = torch.zeros(D, self.Kp)
        conv[:, :k] = _t(sd["visual.conv1.weight"]).float().reshape(D, k)
        head = [f32(sd["visual.ln_pre.weight"]), f32(sd["visual.ln_pre.bias"]),
                f32(sd["visual.ln_post.weight"]), f32(sd["visual.ln_post.bias"]),
                _t(sd["visual.proj"]).float().t().contiguous().to(self.dev, act),
                conv.to(self.dev, act).contiguous(), f32(sd["visual.class_embedding"]),
                f32(sd["visual.positional_embedding"])]
        self._keep = [t for t in table if t is not None] + head
        h = ctypes.c_void_p()
        N.check(N.load().clipk_vision_create(D, nl, D // 64, arch.embed_dim, arch.image_resolution, p,
                                             ops.DT[act], _ptrs(table), _ptrs(head), ctypes.byref(h)),
                "clipk_vision_create")
        self.handle = h

    def forward(self, image):
        if image.requires_grad:
            raise RuntimeError("the image encoder is frozen and forward-only (no input grad)")
        image = image.to(self.dev, torch.float32).contiguous()
        B = image.shape[0]
        if image.shape[1:] != (3, self.input_resolution, self.input_resolution):
            raise RuntimeError(f"expected [B,3,{self.input_resolution},{self.input_resolution}] images, "
                               f"got {tuple(image.shape)}")
        lib = N.load()
        feat = torch.empty(B, self.output_dim, device=self.dev)
        wsb = lib.clipk_vit_ws_bytes(self.handle, B)
        ws = WORKSPACE.get(wsb, self.dev, "vit")
        N.check(lib.clipk_vit_forward(self.handle, B, ops._p(image), ops._p(feat), ops._p(ws), ws.numel(),
                                      ops._stream()), "clipk_vit_forward")
        return feat

    def __del__(self):
        _Encoder.__del__(self)


class CLIP(nn.Module):
    """Container with the attributes the prompt learners read (model.py:488-561)."""

    def __init__(self, sd, prec: str = "fp16", device="cuda", text_grad: bool = True):
        super().__init__()
        if prec not in PREC_DTYPES:
            raise AssertionError(f"PREC must be one of {list(PREC_DTYPES)}")
        arch = arch_from_state_dict(sd)
        self.arch, self.prec = arch, prec
        dev = torch.device(device)
        self.visual = VisionEncoder(sd, arch, prec, dev)
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


def build_model(state_dict, prec: str = "fp16", device="cuda", text_grad: bool = True) -> CLIP:
    """build_model(state_dict) analogue (model.py:662-705) for the native path."""
    return CLIP(state_dict, prec=prec, device=device, text_grad=text_grad)
