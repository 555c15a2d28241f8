"""The image encoder beside the text encoder, on vs off, interleaved on one box:
CoOp (NATIVE.OVERLAP_VISION: the ViT on a side stream beside the image-independent text
encoder; NATIVE.PREFETCH_VISION: the next batch's ViT on a side stream for the whole step and
the post-step accuracy forward reusing the step's features; BASELINE config 2: ViT-B/16 fp16,
n_ctx 16, 1,000 classes, batch 32) and CoCoOp
(NATIVE.PREFETCH_VISION: the next batch's ViT on a side stream for the whole step; the
headline: 8 images, and the reference's batch of 1)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arch", default="ViT-B/16")
    ap.add_argument("--prec", default="fp16")
    ap.add_argument("--classes", type=int, default=1000)
    ap.add_argument("--trainer", default="both", choices=["coop", "cocoop", "both"])
    a = ap.parse_args()
    import torch
    import bench
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    coop_sets = (("overlap+prefetch", {"OVERLAP_VISION": True, "PREFETCH_VISION": True}),
                 ("overlap", {"OVERLAP_VISION": True, "PREFETCH_VISION": False}),
                 ("inline", {"OVERLAP_VISION": False, "PREFETCH_VISION": False}))
    cocoop_sets = (("prefetch", {"PREFETCH_VISION": True}), ("inline", {"PREFETCH_VISION": False}))
    runs = []
    if a.trainer in ("coop", "both"):
        runs.append(("CoOp batch 32", coop_sets, 32, bench.build_coop_trainer(a, a.prec, 32, dev, 0)))
    if a.trainer in ("cocoop", "both"):
        for b in (8, 1):
            runs.append((f"CoCoOp batch {b}", cocoop_sets, b, bench.build_trainer(a, a.prec, b, dev, 0)))
    for name, sets, b, (tr, dm) in runs:
        for rnd in range(2):
            for tag, knobs in sets:
                tr.cfg.NATIVE.update(knobs)
                t, _ = bench.time_train(tr, dm, 20, 3)
                print(f"{name} round {rnd} {tag}: {t / 20 * 1e3:.3f} ms/step, {b * 20 / t:.1f} images/s")

if __name__ == "__main__":
    main()
