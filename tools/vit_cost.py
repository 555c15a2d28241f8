"""What the side-stream ViT costs the CoCoOp train step: step time as usual vs with the image
encoder replaced by a cached-features stub (same shapes, no ViT kernels), interleaved.
    python tools/vit_cost.py [--batch 8] [--steps 40]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--arch", default="ViT-B/16")
    ap.add_argument("--classes", type=int, default=1000)
    ap.add_argument("--prec", default="fp16")
    a = ap.parse_args()
    import torch
    import bench
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    tr, dm = bench.build_trainer(a, a.prec, a.batch, dev, 0)
    m = tr.model
    real = m.image_encoder
    with torch.no_grad():
        feats = {id(b["img"]): real(b["img"]).clone() for b in dm.train_loader_x}
    torch.cuda.synchronize()
    class Stub(torch.nn.Module):
        def forward(self, img):
            return feats[id(img)]
    stub = Stub()
    res = {"batch": a.batch}
    for mode in ("vit", "stub", "vit", "stub"):
        m.image_encoder = real if mode == "vit" else stub
        t, _ = bench.time_train(tr, dm, a.steps, 5)
        res.setdefault(mode, []).append(round(1e3 * t / a.steps, 4))
    m.image_encoder = real
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
