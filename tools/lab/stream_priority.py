"""Does running the train step's main stream at high priority (the side-stream ViT at normal
priority) shorten the step? The CoCoOp bench step on the default stream vs inside a
torch.cuda.Stream(priority=<highest>) made current for the whole loop, interleaved, two rounds.
    PREC=fp32s python tools/lab/stream_priority.py [8/1000,1/1000]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    cases = sys.argv[1] if len(sys.argv) > 1 else "8/1000,1/1000"
    prec = os.environ.get("PREC", "fp32s")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    lo, hi = torch.cuda.Stream.priority_range() if hasattr(torch.cuda.Stream, "priority_range") else (0, -1)
    print(f"priority range (low, high): {lo}, {hi}", flush=True)
    hp = torch.cuda.Stream(device=dev, priority=hi)
    for tok in cases.split(","):
        b, c = (int(x) for x in tok.split("/"))
        tr, dm = bench.build_trainer(argparse.Namespace(arch="ViT-B/16", classes=c), prec, b, dev, 0)
        n = 50 if b == 1 else 20
        res = {"default": [], "high": []}
        for _ in range(2):
            res["default"].append(1000 * bench.time_train(tr, dm, n, 5)[0] / n)
            torch.cuda.synchronize()
            with torch.cuda.stream(hp):
                res["high"].append(1000 * bench.time_train(tr, dm, n, 5)[0] / n)
            torch.cuda.synchronize()
        print(f"{prec} B {b} C {c:5d}: " + "  ".join(f"{k} " + " ".join(f"{t:.3f}" for t in v)
                                                   for k, v in res.items()) + " ms/step", flush=True)
        del tr, dm
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
