"""GPU preprocessing (csrc/preprocess.hip through the C-ABI) vs the reference's transform
chain executed with Pillow + torch on the CPU: Resize(shorter edge, BICUBIC) -> CenterCrop
for test, crop -> resize(BICUBIC) -> horizontal flip for train, then ToTensor
(float().div(255)) and Normalize(sub_(mean).div_(std)). Bit-exact: resampled uint8 pixels
equal, normalised fp32 tensors equal."""
import numpy as np
import pytest
import torch
from PIL import Image

from fsp_amd.data import preprocess as P

pytestmark = pytest.mark.gpu


def _ref(img, plan):
    im = Image.fromarray(img)
    if (plan.x0, plan.y0, plan.w, plan.h) != (0, 0) + im.size:
        im = im.crop((plan.x0, plan.y0, plan.x0 + plan.w, plan.y0 + plan.h))  # RandomResizedCrop window
    im = im.resize((plan.rw, plan.rh), Image.BICUBIC)  # a same-size resize is a copy
    im = im.crop((plan.ox, plan.oy, plan.ox + plan.S, plan.oy + plan.S))  # CenterCrop (test)
    if plan.flip:
        im = im.transpose(Image.FLIP_LEFT_RIGHT)
    a = np.asarray(im)
    t = torch.from_numpy(a.copy()).permute(2, 0, 1).contiguous()
    x = t.float().div(255)
    m = torch.tensor(P.MEAN, dtype=torch.float32)[:, None, None]
    s = torch.tensor(P.STD, dtype=torch.float32)[:, None, None]
    return t, x.sub_(m).div_(s)


def _images(seed, n):
    rs = np.random.RandomState(seed)
    return [rs.randint(0, 256, size=(int(rs.randint(60, 700)), int(rs.randint(60, 700)), 3), dtype=np.uint8)
            for _ in range(n)]


@pytest.mark.parametrize("train", [False, True])
def test_preprocess_matches_pillow_pipeline(dev, train):
    imgs = _images(11 if train else 7, 12)
    g = torch.Generator().manual_seed(5)
    plans = [P.train_plan(im.shape[1], im.shape[0], 224, generator=g) if train else
             P.test_plan(im.shape[1], im.shape[0], 224) for im in imgs]
    if train:
        plans[0].flip = True
    out8 = P.preprocess_batch(imgs, plans, device=str(dev), out_uint8=True).cpu()
    out = P.preprocess_batch(imgs, plans, device=str(dev)).cpu()
    for b, (im, p) in enumerate(zip(imgs, plans)):
        r8, rf = _ref(im, p)
        assert torch.equal(out8[b], r8), (b, (out8[b].int() - r8.int()).abs().max())
        assert torch.equal(out[b], rf), b


def test_gpu_transform_cfg_surface(dev):
    from fsp_amd.engine.config import get_cfg_default
    cfg = get_cfg_default()
    cfg.INPUT.SIZE = (224, 224)
    cfg.INPUT.TRANSFORMS = ["random_resized_crop", "random_flip", "normalize"]
    cfg.INPUT.INTERPOLATION = "bicubic"
    tf = P.GpuTransform(cfg, is_train=True, device=str(dev))
    x = tf(_images(3, 4))
    assert x.shape == (4, 3, 224, 224) and x.dtype == torch.float32 and torch.isfinite(x).all()
    te = P.GpuTransform(cfg, is_train=False, device=str(dev))
    imgs = _images(4, 3)
    y = te(imgs)
    for b, im in enumerate(imgs):
        assert torch.equal(y[b].cpu(), _ref(im, P.test_plan(im.shape[1], im.shape[0], 224))[1])
