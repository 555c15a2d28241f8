"""PREC fp32s headline line (CoCoOp ViT-B/16, C = 1000, B = 8) on fp16-valued weights (split mode 2,
CLIPK_F32S16) and on fp32-valued weights (mode 1), two interleaved rounds each.
    python tools/lab/fp32s_w16.py"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import torch
    import bench
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    base = dict(arch="ViT-B/16", classes=1000, batch=8)
    for rnd in range(2):
        for w in ("fp16", "fp32"):
            args = argparse.Namespace(**base, weights=w)
            line = bench.precision_line(args, "fp32s", dev, 0, 1, n_eval=2000, prof=rnd == 0)
            print(json.dumps({"round": rnd, "weights": w, **line}), flush=True)


if __name__ == "__main__":
    main()
