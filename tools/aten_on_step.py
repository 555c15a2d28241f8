"""Which non-clipk GPU kernels a headline train step launches, and from where (torch.profiler
with Python stacks): bench.py's trainer, 3 warm-up steps, then 2 profiled steps.

    python tools/aten_on_step.py [--prec fp32s] [--batch 8] [--classes 1000]"""
import argparse
import os
import sys
from collections import Counter, defaultdict

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--prec", default="fp32s")
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--classes", type=int, default=1000)
    a = ap.parse_args()
    args = argparse.Namespace(arch="ViT-B/16", classes=a.classes, weights="fp16", batch=a.batch)
    dev = torch.device("cuda", 0)
    tr, dm = bench.build_trainer(args, a.prec, a.batch, dev, 0)
    batches = dm.train_loader_x

    def step(i):
        tr.batch_idx = i
        tr.next_batch = batches[(i + 1) % len(batches)]
        tr.forward_backward(batches[i % len(batches)])
    for i in range(3):
        step(i)
    torch.cuda.synchronize()
    from torch.profiler import profile, ProfilerActivity
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
        for i in range(2):
            step(i)
        torch.cuda.synchronize()
    kern = Counter()
    where = defaultdict(Counter)
    for ev in prof.events():
        if ev.device_type != torch.autograd.DeviceType.CUDA:
            continue
        n = ev.name
        if "clipk" in n:
            continue
        kern[n[:110]] += 1
    # CPU ops that launched kernels: aten ops with a CUDA child
    for ev in prof.events():
        if ev.device_type == torch.autograd.DeviceType.CUDA or not ev.name.startswith("aten::"):
            continue
        ks = getattr(ev, "kernels", None) or []
        if not any("clipk" not in k.name for k in ks):
            continue
        st = [f for f in (ev.stack or []) if "fsp_amd" in f or "few-shot" in f or "bench.py" in f]
        where[ev.name][st[0] if st else "?"] += 1
    print("non-clipk GPU kernels over 2 steps:")
    for k, c in kern.most_common():
        print(f"  {c:4d}  {k}")
    print("aten ops launching them (first repo frame):")
    for op, cs in where.items():
        for s, c in cs.most_common(4):
            print(f"  {c:4d}  {op:40s} {s}")


if __name__ == "__main__":
    main()
