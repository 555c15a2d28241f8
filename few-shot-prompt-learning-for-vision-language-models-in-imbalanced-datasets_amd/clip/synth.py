"""Seeded synthetic CLIP state dicts and inputs (no network, no checkpoints).

The reference loads OpenAI CLIP checkpoints by URL (``PromptSRC/clip/clip.py:39-68``),
which is impossible offline, so parity and benchmarks run on random weights that
follow the reference's own init stds (``PromptSRC/clip/model.py:563-590``) drawn from
``numpy.random.RandomState`` (legacy stream: version-stable, so the fixtures made in
the survey container regenerate bit-identically on the GPU box).

Key layout follows the CLIP state dict that ``build_model`` consumes
(``PromptSRC/clip/model.py:662-705``): ``visual.*``, ``transformer.resblocks.i.*``,
``token_embedding.weight``, ``positional_embedding``, ``ln_final.*``,
``text_projection``, ``logit_scale``.

Deviation from a pure reference init (documented in DESIGN.md): biases and LayerNorm
affine parameters are drawn non-trivially (bias ~ N(0, 0.02), LN gamma ~ 1 + N(0, 0.05),
LN beta ~ N(0, 0.02)) so that parity tests exercise every parameter; the reference
would leave MHA biases at 0 and LN at (1, 0).
"""
from __future__ import annotations

import hashlib
from dataclasses import dataclass, asdict

import numpy as np

CLIP_MEAN = (0.48145466, 0.4578275, 0.40821073)
CLIP_STD = (0.26862954, 0.26130258, 0.27577711)


@dataclass(frozen=True)
class ClipArch:
    embed_dim: int
    image_resolution: int
    vision_layers: int
    vision_width: int
    vision_patch_size: int
    context_length: int
    vocab_size: int
    transformer_width: int
    transformer_heads: int
    transformer_layers: int

    @property
    def vision_heads(self) -> int:  # model.py:506 (ViT branch)
        return self.vision_width // 64

    @property
    def grid(self) -> int:
        return self.image_resolution // self.vision_patch_size

    @property
    def image_tokens(self) -> int:
        return self.grid * self.grid + 1

    def as_dict(self):
        return asdict(self)


ARCHS = {
    "ViT-B/32": ClipArch(512, 224, 12, 768, 32, 77, 49408, 512, 8, 12),
    "ViT-B/16": ClipArch(512, 224, 12, 768, 16, 77, 49408, 512, 8, 12),
    "ViT-L/14": ClipArch(768, 224, 24, 1024, 14, 77, 49408, 768, 12, 12),
    "ViT-L/14@336px": ClipArch(768, 336, 24, 1024, 14, 77, 49408, 768, 12, 12),
    # Small shapes for exhaustive parity (every width a multiple of 128, head dim 64).
    "tiny": ClipArch(128, 32, 2, 128, 16, 77, 49408, 128, 2, 2),
    "tiny-p8": ClipArch(128, 32, 2, 128, 8, 77, 49408, 128, 2, 2),
    "tiny4": ClipArch(128, 32, 4, 128, 16, 77, 49408, 128, 2, 4),  # deep-prompt depth coverage
}


def _param_specs(a: ClipArch):
    """(key, shape, kind, std) in a FIXED order; kind in {w, b, lnw, lnb, const}."""
    specs = []
    D, W, E = a.vision_width, a.transformer_width, a.embed_dim
    vscale = D ** -0.5  # model.py:386-391
    specs += [
        ("visual.class_embedding", (D,), "w", vscale),
        ("visual.positional_embedding", (a.image_tokens, D), "w", vscale),
        ("visual.proj", (D, E), "w", vscale),
        ("visual.conv1.weight", (D, 3, a.vision_patch_size, a.vision_patch_size), "w",
         (3 * a.vision_patch_size ** 2) ** -0.5),
        ("visual.ln_pre.weight", (D,), "lnw", 0.0),
        ("visual.ln_pre.bias", (D,), "lnb", 0.0),
    ]

    def blocks(prefix, width, layers):
        out = []
        proj_std = (width ** -0.5) * ((2 * layers) ** -0.5)  # model.py:579-581
        attn_std = width ** -0.5
        fc_std = (2 * width) ** -0.5
        for i in range(layers):
            p = f"{prefix}.resblocks.{i}."
            out += [
                (p + "attn.in_proj_weight", (3 * width, width), "w", attn_std),
                (p + "attn.in_proj_bias", (3 * width,), "b", 0.0),
                (p + "attn.out_proj.weight", (width, width), "w", proj_std),
                (p + "attn.out_proj.bias", (width,), "b", 0.0),
                (p + "ln_1.weight", (width,), "lnw", 0.0),
                (p + "ln_1.bias", (width,), "lnb", 0.0),
                (p + "mlp.c_fc.weight", (4 * width, width), "w", fc_std),
                (p + "mlp.c_fc.bias", (4 * width,), "b", 0.0),
                (p + "mlp.c_proj.weight", (width, 4 * width), "w", proj_std),
                (p + "mlp.c_proj.bias", (width,), "b", 0.0),
                (p + "ln_2.weight", (width,), "lnw", 0.0),
                (p + "ln_2.bias", (width,), "lnb", 0.0),
            ]
        return out

    specs += blocks("visual.transformer", D, a.vision_layers)
    specs += [
        ("visual.ln_post.weight", (D,), "lnw", 0.0),
        ("visual.ln_post.bias", (D,), "lnb", 0.0),
        ("token_embedding.weight", (a.vocab_size, W), "w", 0.02),   # model.py:564
        ("positional_embedding", (a.context_length, W), "w", 0.01),  # model.py:565
    ]
    specs += blocks("transformer", W, a.transformer_layers)
    specs += [
        ("ln_final.weight", (W,), "lnw", 0.0),
        ("ln_final.bias", (W,), "lnb", 0.0),
        ("text_projection", (W, E), "w", W ** -0.5),  # model.py:589-590
    ]
    return specs


def make_state_dict(arch: str | ClipArch, seed: int = 0, logit_scale: float = float(np.log(100.0)),
                    fp16_values: bool = False):
    """Return {key: float32 ndarray} for a CLIP model of the given architecture. fp16_values:
    every parameter rounded to fp16 (then stored as float32), as the released CLIP checkpoints
    hold them (fp16 archives, PromptSRC/clip/clip.py:154-180; build_model copies them into the
    fp32 model, model.py:699-701): the weights a real fp32 run multiplies."""
    a = ARCHS[arch] if isinstance(arch, str) else arch
    rs = np.random.RandomState(seed)
    sd = {}
    for key, shape, kind, std in _param_specs(a):
        z = rs.standard_normal(size=shape)
        if kind == "w":
            v = z * std
        elif kind == "b":
            v = z * 0.02
        elif kind == "lnw":
            v = 1.0 + 0.05 * z
        elif kind == "lnb":
            v = 0.02 * z
        else:
            raise AssertionError(kind)
        if fp16_values:
            v = v.astype(np.float16)
        sd[key] = np.ascontiguousarray(v, dtype=np.float32)
    sd["logit_scale"] = np.asarray(logit_scale, dtype=np.float32)
    return sd


def state_dict_digest(sd) -> str:
    """Stable short digest of a state dict (detects generator drift vs fixtures)."""
    h = hashlib.sha256()
    for k in sorted(sd):
        v = np.asarray(sd[k], dtype=np.float32)
        h.update(k.encode())
        h.update(np.ascontiguousarray(v).tobytes())
    return h.hexdigest()[:16]


def make_images(batch: int, resolution: int, seed: int = 1) -> np.ndarray:
    """U[0,1) images, CLIP-normalised, NCHW float32."""
    rs = np.random.RandomState(seed)
    u = rs.random_sample(size=(batch, 3, resolution, resolution)).astype(np.float32)
    mean = np.asarray(CLIP_MEAN, dtype=np.float32)[None, :, None, None]
    std = np.asarray(CLIP_STD, dtype=np.float32)[None, :, None, None]
    return ((u - mean) / std).astype(np.float32)


def make_labels(batch: int, n_cls: int, seed: int = 2) -> np.ndarray:
    rs = np.random.RandomState(seed)
    return rs.randint(0, n_cls, size=(batch,)).astype(np.int64)


def synthetic_classnames(n_cls: int):
    return [f"class{i}" for i in range(n_cls)]


def make_ctx(n_ctx: int, width: int, n_cls: int | None = None, seed: int = 3) -> np.ndarray:
    """Context vectors ~ N(0, 0.02) (coop.py:228-234), [n_ctx,W] or [C,n_ctx,W] (CSC)."""
    rs = np.random.RandomState(seed)
    shape = (n_ctx, width) if n_cls is None else (n_cls, n_ctx, width)
    return (rs.standard_normal(size=shape) * 0.02).astype(np.float32)


def make_meta_net(vis_dim: int, ctx_dim: int, seed: int = 4) -> dict:
    """Meta-Net params (cocoop.py:139-143) ~ U(-1/sqrt(fan_in), 1/sqrt(fan_in))."""
    rs = np.random.RandomState(seed)
    hid = vis_dim // 16

    def u(shape, fan_in):
        b = 1.0 / np.sqrt(fan_in)
        return rs.uniform(-b, b, size=shape).astype(np.float32)

    return {
        "meta_net.linear1.weight": u((hid, vis_dim), vis_dim),
        "meta_net.linear1.bias": u((hid,), vis_dim),
        "meta_net.linear2.weight": u((ctx_dim, hid), hid),
        "meta_net.linear2.bias": u((ctx_dim,), hid),
    }
