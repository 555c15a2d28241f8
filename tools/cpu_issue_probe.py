"""Is the training step GPU-bound? Host time to issue K steps (no synchronisation inside the
loop) against the wall time until the GPU has finished them, for the headline CoCoOp step (8
images) and the reference's batch of 1. issue << total: the host runs ahead of the GPU (GPU-bound);
issue ~ total: the host is the bottleneck."""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arch", default="ViT-B/16")
    ap.add_argument("--classes", type=int, default=1000)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--batches", default="8,1")
    a = ap.parse_args()
    import torch
    import bench
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    tr, dm = bench.build_trainer(a, "fp16", 8, dev, 0)
    for b in (int(x) for x in a.batches.split(",")):
        batches = [{"img": x["img"][:b], "label": x["label"][:b]} for x in dm.train_loader_x]

        def step(i):
            tr.batch_idx = i
            tr.next_batch = batches[(i + 1) % len(batches)]
            return tr.forward_backward(batches[i % len(batches)])

        for i in range(3):
            step(i)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(a.steps):
            step(i)
        t_issue = time.perf_counter() - t0
        torch.cuda.synchronize()
        t_total = time.perf_counter() - t0
        print(f"batch {b}: host issue {t_issue / a.steps * 1e3:.3f} ms/step, wall {t_total / a.steps * 1e3:.3f} "
              f"ms/step", flush=True)


if __name__ == "__main__":
    main()
