"""Train-step time with the step's main-stream work on a high-priority stream (the frozen ViT
prefetch keeps its default-priority side stream) vs the default stream: does queue priority
keep the side-stream ViT from delaying the critical text path?
    python tools/prio_time.py [--batch 8] [--steps 50]"""
import argparse
import json
import os
import sys
import time

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
    lo, hi = torch.cuda.Stream.priority_range() if hasattr(torch.cuda.Stream, "priority_range") else (0, -1)
    hp = torch.cuda.Stream(dev, priority=hi)
    res = {"batch": a.batch, "priority_range": [lo, hi]}
    for mode in ("default", "high", "default", "high"):
        if mode == "high":
            hp.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(hp):
                t, _ = bench.time_train(tr, dm, a.steps, 5)
            torch.cuda.current_stream(dev).wait_stream(hp)
        else:
            t, _ = bench.time_train(tr, dm, a.steps, 5)
        res.setdefault(mode, []).append(round(1e3 * t / a.steps, 4))
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
