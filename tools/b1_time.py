"""CoCoOp batch-1 train step (the reference's CoCoOp batch, vit_b16_c4_ep10_batch1_ctxv1.yaml:3)
on one GPU: ms/step over --steps timed steps; knobs come from the environment (A/B runs).
    python tools/b1_time.py [--steps 50] [--batch 1]"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--arch", default="ViT-B/16")
    ap.add_argument("--classes", type=int, default=1000)
    ap.add_argument("--prec", default="fp16")
    a = ap.parse_args()
    import torch
    import bench
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    tr, dm = bench.build_trainer(a, a.prec, a.batch, dev, 0)
    t, _ = bench.time_train(tr, dm, a.steps, 5)
    knobs = {k: v for k, v in os.environ.items() if k.startswith("CLIPK_")}
    print(json.dumps({"batch": a.batch, "ms_per_step": round(1e3 * t / a.steps, 4), "knobs": knobs}), flush=True)


if __name__ == "__main__":
    main()
