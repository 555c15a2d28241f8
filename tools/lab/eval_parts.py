"""Eval (forward-only, test batch 100) of the CoCoOp bench configuration over N images, meant to
run under `rocprofv3 --kernel-trace --stats` to see where eval time goes.
    PREC=fp32s python tools/lab/eval_parts.py [images]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
    prec = os.environ.get("PREC", "fp32s")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    tr, dm = bench.build_trainer(argparse.Namespace(arch="ViT-B/16", classes=1000), prec, 8, dev, 0,
                                 n_test=min(n, 1000))
    rate, imgs = bench.time_eval(tr, dm, n)
    print(f"{prec} eval: {rate:.1f} images/s over {imgs} images ({1000.0 / rate:.3f} ms per image)", flush=True)


if __name__ == "__main__":
    main()
