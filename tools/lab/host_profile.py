"""Where the host time of a batch-1 train step goes: cProfile over 50 steps of the bench loop
(bench.time_train's step, after warm-up), top functions by own time and by cumulative time.
    python tools/lab/host_profile.py [classes]"""
import argparse
import cProfile
import io
import os
import pstats
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    c = int(sys.argv[1]) if len(sys.argv) > 1 else 125
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    tr, dm = bench.build_trainer(argparse.Namespace(arch="ViT-B/16", classes=c), "fp16", 1, dev, 0)
    bl = dm.train_loader_x

    def steps(n):
        for i in range(n):
            tr.batch_idx = i
            tr.next_batch = bl[(i + 1) % len(bl)]
            tr.forward_backward(bl[i % len(bl)])

    steps(10)
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    pr.enable()
    steps(50)
    pr.disable()
    torch.cuda.synchronize()
    for key in ("tottime", "cumulative"):
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats(key).print_stats(30)
        print(s.getvalue(), flush=True)


if __name__ == "__main__":
    main()
