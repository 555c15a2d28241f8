"""Host half of the GPU preprocessing: the fixed-point bicubic coefficient tables
(fsp_amd/data/preprocess.py, restating Pillow's Resample.c) reproduce Pillow's own
Image.resize(BICUBIC) bit-exactly when applied with Pillow's integer two-pass scheme
(numpy here; the HIP kernels do the same integer work on the GPU, tests/test_preprocess_gpu.py).
Pillow is the library the reference's torchvision transforms call (transforms.py:206-354)."""
import numpy as np
import pytest
from PIL import Image

from fsp_amd.data import preprocess as P


def _apply(img, x0, y0, w, h, rw, rh):
    """Pillow two-pass resample of window (x0, y0, w, h) to (rw, rh) with our tables."""
    hx, hn, hk = P.resample_coeffs(w, rw)
    vy, vn, vk = P.resample_coeffs(h, rh)
    ty0, ty1 = int(vy.min()), int((vy + vn).max())
    src = img[y0 + ty0:y0 + ty1, x0:x0 + w].astype(np.int64)
    tmp = np.empty((ty1 - ty0, rw, 3), np.int64)
    half = 1 << (P.PRECISION_BITS - 1)
    for x in range(rw):
        taps = src[:, hx[x]:hx[x] + hn[x]]
        tmp[:, x] = np.clip((half + (taps * hk[x, :hn[x], None]).sum(1)) >> P.PRECISION_BITS, 0, 255)
    out = np.empty((rh, rw, 3), np.int64)
    for y in range(rh):
        taps = tmp[vy[y] - ty0:vy[y] - ty0 + vn[y]]
        out[y] = np.clip((half + (taps * vk[y, :vn[y], None, None]).sum(0)) >> P.PRECISION_BITS, 0, 255)
    return out.astype(np.uint8)


@pytest.mark.parametrize("H,W,rw,rh", [(37, 53, 224, 224), (500, 375, 224, 298), (640, 480, 299, 224),
                                       (224, 224, 224, 224), (97, 301, 64, 17)])
def test_tables_match_pillow_resize(H, W, rw, rh):
    rs = np.random.RandomState(H * 7 + W)
    img = rs.randint(0, 256, size=(H, W, 3), dtype=np.uint8)
    ref = np.asarray(Image.fromarray(img).resize((rw, rh), Image.BICUBIC))
    assert np.array_equal(_apply(img, 0, 0, W, H, rw, rh), ref)


def test_crop_window_matches_pillow_crop_then_resize():
    rs = np.random.RandomState(3)
    img = rs.randint(0, 256, size=(333, 444, 3), dtype=np.uint8)
    x0, y0, w, h = 57, 31, 201, 260
    ref = np.asarray(Image.fromarray(img).crop((x0, y0, x0 + w, y0 + h)).resize((224, 224), Image.BICUBIC))
    assert np.array_equal(_apply(img, x0, y0, w, h, 224, 224), ref)


def test_geometry_helpers():
    assert P.shorter_edge_size(500, 375, 224) == (298, 224)
    assert P.shorter_edge_size(375, 500, 224) == (224, 298)
    assert P.shorter_edge_size(224, 300, 224) == (224, 300)
    assert P.center_crop_origin(298, 224, 224, 224) == (37, 0)
    assert P.center_crop_origin(225, 224, 224, 224) == (0, 0)  # round(0.5) == 0 (half to even)
    import torch
    g = torch.Generator().manual_seed(0)
    for _ in range(50):
        i, j, h, w = P.rrc_params(500, 375, generator=g)
        assert 0 <= i and i + h <= 375 and 0 <= j and j + w <= 500 and h > 0 and w > 0
