"""Throughput of the GPU preprocessing (test and train transforms, 224x224 out) on a batch
of decoded 500x375 uint8 images already resident on the device, vs the same transforms with
Pillow + torch on one host core (the reference's per-image DataLoader work)."""
import os
import sys
import time

import numpy as np
import torch
from PIL import Image

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fsp_amd.data import preprocess as P  # noqa: E402


def main():
    B = int(os.environ.get("PB_B", 256))
    rs = np.random.RandomState(0)
    imgs = [rs.randint(0, 256, size=(375, 500, 3), dtype=np.uint8) for _ in range(B)]
    dev_imgs = [torch.from_numpy(im).cuda() for im in imgs]
    for train in (False, True):
        g = torch.Generator().manual_seed(0)
        plans = [P.train_plan(500, 375, 224, generator=g) if train else P.test_plan(500, 375, 224) for _ in imgs]
        P.preprocess_batch(dev_imgs, plans)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(10):
            P.preprocess_batch(dev_imgs, plans)
        torch.cuda.synchronize()
        gpu = 10 * B / (time.perf_counter() - t0)
        t0 = time.perf_counter()
        n = 32
        for im, p in zip(imgs[:n], plans[:n]):
            x = Image.fromarray(im)
            if train:
                x = x.crop((p.x0, p.y0, p.x0 + p.w, p.y0 + p.h))
            x = x.resize((p.rw, p.rh), Image.BICUBIC).crop((p.ox, p.oy, p.ox + 224, p.oy + 224))
            t = torch.from_numpy(np.asarray(x).copy()).permute(2, 0, 1).float().div(255)
            t.sub_(torch.tensor(P.MEAN)[:, None, None]).div_(torch.tensor(P.STD)[:, None, None])
        cpu = n / (time.perf_counter() - t0)
        print(f"{'train' if train else 'test '} transform: GPU {gpu:9.1f} img/s (incl. host plan/tables, "
              f"batch {B}) | Pillow+torch 1 core {cpu:7.1f} img/s")


if __name__ == "__main__":
    torch.set_num_threads(1)
    main()
