"""Per-launch-site times (HIP events around every named encoder launch) of one workload's train
step: python tools/site_table.py --arch ViT-L/14@336px --prec bf16 [--batch 8]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arch", default="ViT-B/16")
    ap.add_argument("--prec", default="fp16")
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--classes", type=int, default=1000)
    a = ap.parse_args()
    import torch
    import bench
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    tr, dm = bench.build_trainer(a, a.prec, a.batch, dev, 0)
    _, sites = bench.time_train(tr, dm, 3, 2, prof_steps=3)
    tot = sum(v[0] for v in sites.values()) / 3
    print(f"sum of sites {tot:.3f} ms/step")
    for name, v in sorted(sites.items(), key=lambda kv: -kv[1][0]):
        ms, n, fl, by = v[0] / 3, v[1] / 3, v[2] / 3, v[3] / 3
        print(f"{name:28s} {ms:7.3f} ms/step {n:5.0f} launches  {fl / ms / 1e9 if ms else 0:7.1f} TF/s  "
              f"{by / ms / 1e6 if ms else 0:7.1f} GB/s")


if __name__ == "__main__":
    main()
