"""Which side stream the ViT prefetch gets: torch hands out pool streams round-robin and HIP
places each stream on one of GPU_MAX_HW_QUEUES hardware queues, so a side stream can land on
the main stream's queue and serialise behind it. Per candidate stream (8 consecutive pool
streams at normal priority, 2 at high priority): the train step with the trainer's side stream
set to it.
    python tools/lab/side_stream_ab.py [batch] [prec]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    b = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    prec = sys.argv[2] if len(sys.argv) > 2 else "fp16"
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    tr, dm = bench.build_trainer(argparse.Namespace(arch="ViT-B/16", classes=1000), prec, b, dev, 0)
    n = 50 if b == 1 else (10 if prec != "fp16" else 20)
    cands = [("pool", i, torch.cuda.Stream(device=dev)) for i in range(8)]
    cands += [("high", i, torch.cuda.Stream(device=dev, priority=-1)) for i in range(2)]
    for rnd in range(2):
        line = f"{prec} B {b} round {rnd}:"
        for kind, i, s in cands:
            tr.model._side_stream = s
            t = bench.time_train(tr, dm, n, 3)[0]
            line += f" {kind}{i} {1000 * t / n:.3f}"
        print(line + " ms/step", flush=True)


if __name__ == "__main__":
    main()
