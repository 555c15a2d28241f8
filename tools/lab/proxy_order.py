"""Why the batch-1 class-shard proxy at 125 classes reads 2.3 ms inside the default bench run and
1.66 ms alone (profiles/r05k, r05n): trainers built one after another in one process, in a given
order, each timed over 50 steps twice (bench.time_train). A token is classes[/batch[/prec[/arch]]],
default batch 1, fp16, ViT-B/16.
    python tools/lab/proxy_order.py 125,1000/8/fp32s,125,1000/32/bf16/ViT-L/14,125"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    import torch
    import bench
    order = sys.argv[1] if len(sys.argv) > 1 else "125,1000,125"
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    for tok in order.split(","):
        f = tok.split("/", 3)
        c, b = int(f[0]), int(f[1]) if len(f) > 1 else 1
        prec = f[2] if len(f) > 2 else "fp16"
        arch = f[3] if len(f) > 3 else "ViT-B/16"
        args = argparse.Namespace(arch=arch, classes=c, prec=prec)
        tr, dm = bench.build_trainer(args, prec, b, dev, 0)
        n = 50 if b == 1 else 10
        ts = [bench.time_train(tr, dm, n, 5)[0] for _ in range(2)]
        print(f"{arch} {prec} B {b} classes {c:5d}: " + " ".join(f"{1000 * t / n:.3f}" for t in ts) + " ms/step",
              flush=True)
        del tr, dm
        if os.environ.get("GC"):
            import gc
            gc.collect()
        torch.cuda.empty_cache()
        print(f"   after del: {torch.cuda.memory_allocated() / 2**20:.0f} MiB allocated, "
              f"{torch.cuda.memory_reserved() / 2**20:.0f} MiB reserved", flush=True)


if __name__ == "__main__":
    main()
