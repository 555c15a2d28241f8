"""What the CoCoOp train step pays for its parts (diagnostic variants, NOT valid bench lines):
  full       the bench step (side-stream ViT of the next batch, PREC fp32s status read per backward)
  no_vit     the image encoder replaced by cached features (the ViT's cost to the step)
  no_sync    the fp32s backward's overflow-flag read skipped (the host synchronisation's cost)
  neither    both
bench.time_train for each, interleaved, two rounds.
    PREC=fp32s python tools/lab/step_parts.py [8/1000,1/1000]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    from fsp_amd.clip import model as M
    cases = sys.argv[1] if len(sys.argv) > 1 else "8/1000,1/1000"
    prec = os.environ.get("PREC", "fp32s")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    real_check = M.TextEncoderCore._check_status
    for tok in cases.split(","):
        b, c = (int(x) for x in tok.split("/"))
        tr, dm = bench.build_trainer(argparse.Namespace(arch="ViT-B/16", classes=c), prec, b, dev, 0)
        model = tr.model
        enc = model.image_encoder
        with torch.no_grad():
            feats = enc(dm.train_loader_x[0]["img"][:b].to(dev))
        class Cached(torch.nn.Module):
            def forward(self, x):
                return feats
        cached = Cached()
        n = 50 if b == 1 else 20
        res = {}
        for _ in range(2):
            for name in ("full", "no_vit", "no_sync", "neither"):
                no_vit = name in ("no_vit", "neither")
                no_sync = name in ("no_sync", "neither")
                model.image_encoder = cached if no_vit else enc
                tr.cfg.NATIVE["PREFETCH_VISION"] = not no_vit
                M.TextEncoderCore._check_status = (lambda self: False) if no_sync else real_check
                res.setdefault(name, []).append(1000 * bench.time_train(tr, dm, n, 5)[0] / n)
        M.TextEncoderCore._check_status = real_check
        model.image_encoder = enc
        print(f"{prec} B {b} C {c:5d}: " + "  ".join(f"{k} " + " ".join(f"{t:.3f}" for t in v)
                                                   for k, v in res.items()) + " ms/step", flush=True)
        del tr, dm, model, enc
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
