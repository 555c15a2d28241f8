"""Is the batch-1 train step bound by the host's launch rate? Per class count: the step's wall
time over 50 steps (synchronised at the ends) against the host time spent inside
forward_backward (no synchronisation per step; the GPU runs behind). Host time close to the wall
time means the GPU waits for launches.
    python tools/lab/host_time.py [125,1000]"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    for c in (int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "125,1000").split(",")):
        tr, dm = bench.build_trainer(argparse.Namespace(arch="ViT-B/16", classes=c), "fp16", 1, dev, 0)
        bl = dm.train_loader_x
        for rnd in range(2):
            for i in range(5):
                tr.batch_idx = i
                tr.next_batch = bl[(i + 1) % len(bl)]
                tr.forward_backward(bl[i % len(bl)])
            torch.cuda.synchronize()
            host = 0.0
            t0 = time.perf_counter()
            for i in range(50):
                tr.batch_idx = i
                tr.next_batch = bl[(i + 1) % len(bl)]
                h0 = time.perf_counter()
                tr.forward_backward(bl[i % len(bl)])
                host += time.perf_counter() - h0
            torch.cuda.synchronize()
            wall = time.perf_counter() - t0
            print(f"classes {c:5d} round {rnd}: wall {wall / 50 * 1e3:.3f} ms/step, host inside forward_backward "
                  f"{host / 50 * 1e3:.3f} ms/step", flush=True)
        del tr, dm
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
