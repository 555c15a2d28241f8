"""CoOp train step with the image encoder on a side stream (NATIVE.OVERLAP_VISION) vs in line,
interleaved on one box (BASELINE config 2: ViT-B/16 fp16, n_ctx 16, 1,000 classes, batch 32;
--arch ViT-L/14 --prec bf16 for config 4)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arch", default="ViT-B/16")
    ap.add_argument("--prec", default="fp16")
    ap.add_argument("--classes", type=int, default=1000)
    ap.add_argument("--batch", type=int, default=32)
    a = ap.parse_args()
    import torch
    import bench
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    tr, dm = bench.build_coop_trainer(a, a.prec, a.batch, dev, 0)
    for rnd in range(2):
        for ov in (True, False):
            tr.cfg.NATIVE.OVERLAP_VISION = ov
            t, _ = bench.time_train(tr, dm, 20, 3)
            print(f"round {rnd} overlap {ov}: {t / 20 * 1e3:.3f} ms/step, {a.batch * 20 / t:.1f} images/s")


if __name__ == "__main__":
    main()
