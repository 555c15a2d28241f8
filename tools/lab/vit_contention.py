"""Which main-stream kernels the side-stream ViT slows: K CoCoOp bench steps with the ViT
prefetch (MODE=vit, the bench step) or with the image encoder replaced by cached features
(MODE=novit, a diagnostic) or with the ViT run in line on the main stream (MODE=serial), meant to run under `rocprofv3 --kernel-trace --stats` once per mode;
compare the per-kernel totals of the two summaries.
    MODE=vit PREC=fp32s [BATCH=8] python tools/lab/vit_contention.py [steps]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    prec = os.environ.get("PREC", "fp32s")
    mode = os.environ.get("MODE", "vit")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    batch = int(os.environ.get("BATCH", "8"))
    tr, dm = bench.build_trainer(argparse.Namespace(arch="ViT-B/16", classes=1000), prec, batch, dev, 0)
    if mode == "novit":
        enc = tr.model.image_encoder
        with torch.no_grad():
            feats = enc(dm.train_loader_x[0]["img"].to(dev))

        class Cached(torch.nn.Module):
            def forward(self, x):
                return feats
        tr.model.image_encoder = Cached()
        tr.cfg.NATIVE["PREFETCH_VISION"] = False
    elif mode == "serial":
        tr.cfg.NATIVE["PREFETCH_VISION"] = False
    t, _ = bench.time_train(tr, dm, steps, 3)
    print(f"{prec} {mode}: {1000 * t / steps:.3f} ms/step over {steps} steps", flush=True)


if __name__ == "__main__":
    main()
