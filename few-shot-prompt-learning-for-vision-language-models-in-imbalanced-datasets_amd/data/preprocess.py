"""GPU-side image preprocessing: the Dassl/torchvision transforms the CoOp/CoCoOp configs
use, on decoded uint8 HWC images, as two HIP kernels (csrc/preprocess.hip).

Reference pipeline (Dassl.pytorch/dassl/data/transforms/transforms.py:206-354, INPUT.
INTERPOLATION "bicubic", configs/trainers/CoCoOp/*.yaml):
* test:  Resize(shorter edge -> max(SIZE)) -> CenterCrop(SIZE) -> ToTensor -> Normalize
* train: RandomResizedCrop(SIZE, scale=RRCROP_SCALE) -> RandomHorizontalFlip -> ToTensor
         -> Normalize
torchvision applies these to PIL images, so the resampling is Pillow's
``Image.resize(BICUBIC)``: separable, antialiased (support x scale when shrinking),
horizontal pass first into a uint8 image, 22-bit fixed-point coefficients
(Pillow libImaging/Resample.c: precompute_coeffs, normalize_coeffs_8bpc). The coefficient
tables are computed here on the host in float64 exactly as that C code does; the kernels
do the integer multiply-accumulate, the uint8 rounding/clipping of both passes, the crop
window, the flip and ToTensor/Normalize in fp32 -- bit-exact to the PIL + torch pipeline
(tests/test_preprocess_*.py check against Pillow itself).

Random crop parameters and the flip coin use a torch CPU generator (the transform's own, or
the global one) in torchvision's call order (RandomResizedCrop.get_params,
RandomHorizontalFlip), restated here: torchvision is not installed, so that sequence is
parity-unpinned (documented in DESIGN.md).
"""
from __future__ import annotations

import math

import numpy as np
import torch

from .. import _native as N
from .. import ops

PRECISION_BITS = 32 - 8 - 2
MEAN = (0.48145466, 0.4578275, 0.40821073)  # configs/trainers/CoCoOp/*.yaml INPUT.PIXEL_MEAN
STD = (0.26862954, 0.26130258, 0.27577711)


def _bicubic(x):
    a = -0.5
    x = np.abs(x)
    return np.where(x < 1.0, ((a + 2.0) * x - (a + 3.0)) * x * x + 1,
                    np.where(x < 2.0, (((x - 5) * x + 8) * x - 4) * a, 0.0))


def resample_coeffs(in_size, out_size, in0=0.0, in1=None):
    """Pillow precompute_coeffs + normalize_coeffs_8bpc for the bicubic filter (support 2):
    returns xmin [out], n [out] (taps used), k int32 [out, ksize]."""
    in1 = float(in_size) if in1 is None else float(in1)
    scale = (in1 - in0) / out_size
    filterscale = max(scale, 1.0)
    support = 2.0 * filterscale
    ksize = int(math.ceil(support)) * 2 + 1
    xx = np.arange(out_size, dtype=np.float64)
    center = in0 + (xx + 0.5) * scale
    ss = 1.0 / filterscale
    xmin = np.maximum((center - support + 0.5).astype(np.int64), 0)       # C (int) truncation
    xmax = np.minimum((center + support + 0.5).astype(np.int64), in_size) - xmin
    x = np.arange(ksize, dtype=np.float64)[None, :]
    w = _bicubic((x + xmin[:, None] - center[:, None] + 0.5) * ss)
    w = np.where(x < xmax[:, None], w, 0.0)
    ww = w.sum(axis=1, keepdims=True)
    w = np.where(ww != 0.0, w / np.where(ww != 0.0, ww, 1.0), w)
    k = np.where(w < 0, (-0.5 + w * (1 << PRECISION_BITS)), (0.5 + w * (1 << PRECISION_BITS)))
    k = np.trunc(k).astype(np.int32)  # C (int) conversion truncates toward zero
    return xmin.astype(np.int32), xmax.astype(np.int32), k


def shorter_edge_size(w, h, size):
    """torchvision F.resize(img, int): (ow, oh)."""
    if (w <= h and w == size) or (h <= w and h == size):
        return w, h
    if w < h:
        return size, int(size * h / w)
    return int(size * w / h), size


def center_crop_origin(w, h, cw, ch):
    """torchvision F.center_crop: (left, top) -- Python round() (half to even)."""
    return int(round((w - cw) / 2.0)), int(round((h - ch) / 2.0))


def rrc_params(width, height, scale=(0.08, 1.0), ratio=(3.0 / 4.0, 4.0 / 3.0), generator=None):
    """torchvision RandomResizedCrop.get_params: (i, j, h, w) on torch's CPU RNG."""
    area = height * width
    log_ratio = torch.log(torch.tensor(ratio))
    for _ in range(10):
        target_area = area * torch.empty(1).uniform_(scale[0], scale[1], generator=generator).item()
        aspect = torch.exp(torch.empty(1).uniform_(log_ratio[0], log_ratio[1], generator=generator)).item()
        w = int(round(math.sqrt(target_area * aspect)))
        h = int(round(math.sqrt(target_area / aspect)))
        if 0 < w <= width and 0 < h <= height:
            i = torch.randint(0, height - h + 1, size=(1,), generator=generator).item()
            j = torch.randint(0, width - w + 1, size=(1,), generator=generator).item()
            return i, j, h, w
    in_ratio = float(width) / float(height)
    if in_ratio < min(ratio):
        w = width
        h = int(round(w / min(ratio)))
    elif in_ratio > max(ratio):
        h = height
        w = int(round(h * max(ratio)))
    else:
        w, h = width, height
    return (height - h) // 2, (width - w) // 2, h, w


class Plan:
    """One image's geometry: source window (x0, y0, w, h) resized to (rw, rh), output
    window (ox, oy, S, S) of the resized image, horizontal flip."""

    def __init__(self, x0, y0, w, h, rw, rh, ox, oy, S, flip):
        self.x0, self.y0, self.w, self.h = x0, y0, w, h
        self.rw, self.rh, self.ox, self.oy, self.S, self.flip = rw, rh, ox, oy, S, flip


def test_plan(w, h, size):
    rw, rh = shorter_edge_size(w, h, size)
    ox, oy = center_crop_origin(rw, rh, size, size)
    return Plan(0, 0, w, h, rw, rh, ox, oy, size, False)


def train_plan(w, h, size, scale=(0.08, 1.0), flip_p=0.5, generator=None):
    i, j, ch, cw = rrc_params(w, h, scale, generator=generator)
    flip = bool(torch.rand(1, generator=generator) < flip_p)
    return Plan(j, i, cw, ch, size, size, 0, 0, size, flip)


def _tables(plans, shapes):
    """Per-image descriptors (int64 [B, 16]) + packed coefficient tables (int32)."""
    desc, tabs, tmp_off, tab_off = [], [], 0, 0
    for p, (H, W) in zip(plans, shapes):
        hx, hn, hk = resample_coeffs(p.w, p.rw)
        vy, vn, vk = resample_coeffs(p.h, p.rh)
        hx, hn, hk = hx[p.ox:p.ox + p.S], hn[p.ox:p.ox + p.S], hk[p.ox:p.ox + p.S]
        vy, vn, vk = vy[p.oy:p.oy + p.S], vn[p.oy:p.oy + p.S], vk[p.oy:p.oy + p.S]
        ty0 = int(vy.min())
        ty1 = int((vy + vn).max())
        rows = max(ty1 - ty0, 1)
        hks, vks = hk.shape[1], vk.shape[1]
        h_tab = np.concatenate([hx[:, None], hn[:, None], hk], axis=1).astype(np.int32)
        v_tab = np.concatenate([(vy - ty0)[:, None], vn[:, None], vk], axis=1).astype(np.int32)
        desc.append([0, W, p.x0, p.y0 + ty0, p.S, int(p.flip), tab_off, hks, tab_off + h_tab.size, vks,
                     tmp_off, rows, H, 0, 0, 0])
        tabs += [h_tab.ravel(), v_tab.ravel()]
        tab_off += h_tab.size + v_tab.size
        tmp_off += rows * p.S * 3
    return np.asarray(desc, np.int64), np.concatenate(tabs).astype(np.int32), tmp_off


def preprocess_batch(images, plans, mean=MEAN, std=STD, device="cuda", out_uint8=False):
    """images: list of uint8 HWC (RGB) numpy arrays or CPU/GPU torch tensors; plans: Plan
    per image (all with the same S). Returns fp32 [B, 3, S, S] normalised on `device` (or
    the uint8 resampled pixels [B, 3, S, S] when out_uint8, for bit-exact checks)."""
    dev = torch.device(device)
    S = plans[0].S
    if any(p.S != S for p in plans):
        raise ValueError("all plans must share the output size")
    ts = [torch.as_tensor(im) for im in images]
    for t in ts:
        if t.dtype != torch.uint8 or t.dim() != 3 or t.shape[2] != 3:
            raise ValueError("images must be uint8 [H, W, 3]")
    shapes = [(int(t.shape[0]), int(t.shape[1])) for t in ts]
    for p, (H, W) in zip(plans, shapes):
        if p.x0 < 0 or p.y0 < 0 or p.x0 + p.w > W or p.y0 + p.h > H or p.rw < p.ox + S or p.rh < p.oy + S:
            raise ValueError("plan window outside the image")
    desc, tab, tmp_elems = _tables(plans, shapes)
    offs = np.cumsum([0] + [H * W * 3 for H, W in shapes])
    desc[:, 0] = offs[:-1]
    src = torch.cat([t.reshape(-1) for t in ts]).to(dev, non_blocking=True)
    d_desc = torch.from_numpy(desc).to(dev)
    d_tab = torch.from_numpy(tab).to(dev)
    tmp = torch.empty(max(tmp_elems, 1), dtype=torch.uint8, device=dev)
    B = len(plans)
    out = torch.empty(B, 3, S, S, device=dev, dtype=torch.uint8 if out_uint8 else torch.float32)
    mean_t = torch.tensor(mean, dtype=torch.float32, device=dev)
    std_t = torch.tensor(std, dtype=torch.float32, device=dev)
    rows_max = int(desc[:, 11].max())
    N.call("clipk_image_resample", B, S, rows_max, ops._p(src), ops._p(d_desc), ops._p(d_tab), ops._p(tmp),
           ops._p(mean_t), ops._p(std_t), 1 if out_uint8 else 0, ops._p(out), ops._stream())
    return out


class GpuTransform:
    """Dassl transform_train / transform_test equivalent for the CoOp/CoCoOp configs
    (random_resized_crop + random_flip + normalize / resize + center_crop + normalize)."""

    def __init__(self, cfg, is_train, device="cuda", generator=None):
        choices = list(cfg.INPUT.TRANSFORMS)
        allowed = {"random_resized_crop", "random_flip", "normalize"}
        if is_train and not set(choices) <= allowed:
            raise NotImplementedError(f"GPU transforms implement {sorted(allowed)}, got {choices}")
        if cfg.INPUT.INTERPOLATION != "bicubic":
            raise NotImplementedError("GPU transforms implement bicubic interpolation")
        self.is_train = is_train
        self.size = max(cfg.INPUT.SIZE)
        self.rrc = "random_resized_crop" in choices
        self.flip = "random_flip" in choices
        self.scale = tuple(cfg.INPUT.get("RRCROP_SCALE", (0.08, 1.0)))
        norm = "normalize" in choices
        self.mean = tuple(cfg.INPUT.PIXEL_MEAN) if norm else (0.0, 0.0, 0.0)
        self.std = tuple(cfg.INPUT.PIXEL_STD) if norm else (1.0, 1.0, 1.0)
        self.device = device
        self.generator = generator  # None: torch's global CPU RNG

    def plan(self, w, h):
        if not self.is_train:
            return test_plan(w, h, self.size)
        if self.rrc:
            return train_plan(w, h, self.size, self.scale, 0.5 if self.flip else 0.0, generator=self.generator)
        rw = rh = self.size  # Resize(input_size) when no random crop
        p = Plan(0, 0, w, h, rw, rh, 0, 0, self.size, False)
        if self.flip:
            p.flip = bool(torch.rand(1, generator=self.generator) < 0.5)
        return p

    def __call__(self, images):
        plans = [self.plan(int(im.shape[1]), int(im.shape[0])) for im in images]
        return preprocess_batch(images, plans, self.mean, self.std, self.device)
