"""CoCoOp train step with the next batch's ViT forward on a side stream (NATIVE.PREFETCH_VISION,
the default) against the ViT inline on the main stream, per batch size and class count
(bench.time_train both ways, interleaved, two rounds each).
    python tools/lab/prefetch_ab.py [1/1000,1/125,2/1000,4/1000,8/1000]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    cases = sys.argv[1] if len(sys.argv) > 1 else "1/1000,1/125,2/1000,4/1000,8/1000"
    prec = os.environ.get("PREC", "fp16")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    for tok in cases.split(","):
        b, c = (int(x) for x in tok.split("/"))
        tr, dm = bench.build_trainer(argparse.Namespace(arch="ViT-B/16", classes=c), prec, b, dev, 0)
        n = 50 if b == 1 else 20
        res = {True: [], False: []}
        for _ in range(2):
            for on in (True, False):
                tr.cfg.NATIVE["PREFETCH_VISION"] = on
                res[on].append(1000 * bench.time_train(tr, dm, n, 5)[0] / n)
        print(f"{prec} B {b} C {c:5d}: side-stream prefetch " + " ".join(f"{t:.3f}" for t in res[True]) +
              " | inline " + " ".join(f"{t:.3f}" for t in res[False]) + " ms/step", flush=True)
        del tr, dm
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
