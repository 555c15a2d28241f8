"""Probe: does replaying the CoCoOp train step as a HIP graph (torch.cuda.graph) shorten it?

Warm-up steps run eagerly, one forward_backward is captured (static batch), then eager and
graph steps are timed in the same process (interleaved). Diagnostic only: the graph bakes the
step's host-side scalars (the SGD learning rate) into its kernel arguments.

    python tools/graph_probe.py [--batch 8] [--classes 1000] [--prec fp16]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--classes", type=int, default=1000)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--prec", default="fp16")
    ap.add_argument("--no-graph", action="store_true", help="eager only: same batch vs alternating batches")
    a = ap.parse_args()
    import torch
    import bench
    args = argparse.Namespace(arch="ViT-B/16", classes=a.classes)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    trainer, dm = bench.build_trainer(args, a.prec, a.batch, dev, 0)
    batch = dm.train_loader_x[0]
    for i in range(3):
        trainer.batch_idx = i
        trainer.forward_backward(batch)
    torch.cuda.synchronize()
    if a.no_graph:
        bl = dm.train_loader_x

        def run(n, alt):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(n):
                trainer.batch_idx = i
                trainer.forward_backward(bl[i % len(bl)] if alt else batch)
            torch.cuda.synchronize()
            return (time.perf_counter() - t0) / n * 1e3

        for r in range(2):
            print(f"round {r}: same batch {run(a.steps, False):.3f} ms/step, alternating {run(a.steps, True):.3f}",
                  flush=True)
        t, _ = bench.time_train(trainer, dm, a.steps, 3)
        print(f"bench.time_train on this trainer: {t / a.steps * 1e3:.3f} ms/step", flush=True)
        tr2, dm2 = bench.build_trainer(args, a.prec, a.batch, dev, 0, n_test=1000)
        t, _ = bench.time_train(tr2, dm2, a.steps, 3)
        print(f"bench.time_train on a second trainer (n_test 1000): {t / a.steps * 1e3:.3f} ms/step", flush=True)
        t, _ = bench.time_train(trainer, dm, a.steps, 3)
        print(f"bench.time_train on the first trainer again: {t / a.steps * 1e3:.3f} ms/step", flush=True)
        return 0
    torch.cuda.synchronize()
    host = []
    for _ in range(10):
        t0 = time.perf_counter()
        trainer.forward_backward(batch)
        host.append((time.perf_counter() - t0) * 1e3)
    torch.cuda.synchronize()
    print(f"host time to issue one step (no sync): min {min(host):.3f} ms, median {sorted(host)[5]:.3f} ms",
          flush=True)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for i in range(2):
            trainer.forward_backward(batch)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    try:
        with torch.cuda.graph(g):
            trainer.forward_backward(batch)
    except Exception as e:  # report what breaks capture
        print("capture failed:", repr(e)[:400], flush=True)
        return 1
    torch.cuda.synchronize()

    def eager(n):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            trainer.forward_backward(batch)
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / n * 1e3

    def graph(n):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            g.replay()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / n * 1e3

    for r in range(3):
        print(f"round {r}: eager {eager(a.steps):.3f} ms/step, graph {graph(a.steps):.3f} ms/step", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
