"""Per-launch-site times (HIP events around every named encoder launch) of the eval forward
(test batch 100, CoCoOp ViT-B/16, 1,000 classes): python tools/eval_sites.py [--prec fp16]"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arch", default="ViT-B/16")
    ap.add_argument("--prec", default="fp16")
    ap.add_argument("--classes", type=int, default=1000)
    ap.add_argument("--batches", type=int, default=4)
    a = ap.parse_args()
    a.batch = 8
    import torch
    import bench
    from fsp_amd import _native as N
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    tr, dm = bench.build_trainer(a, a.prec, 8, dev, 0, n_test_device=100 * a.batches)
    e, n = bench.time_eval(tr, dm, 100 * a.batches)
    print(f"eval {e:.1f} img/s over {n} images ({1e5 / e:.2f} ms per 100-image batch)")
    tr.set_model_mode("eval")
    lib = N.load()
    tl = dm.test_loader
    with torch.no_grad():
        torch.cuda.synchronize()
        lib.clipk_prof_sites_enable(1)
        t0 = time.perf_counter()
        for i in range(a.batches):
            tr.model_inference(tl[i % len(tl)]["img"])
        torch.cuda.synchronize()
        t = time.perf_counter() - t0
        sites = N.prof_sites_read()
        lib.clipk_prof_sites_enable(0)
    tot = sum(v[0] for v in sites.values()) / a.batches
    print(f"with site events: {1e3 * t / a.batches:.2f} ms per batch; sum of sites {tot:.3f} ms per batch")
    for name, v in sorted(sites.items(), key=lambda kv: -kv[1][0]):
        ms, cnt, fl, by = (x / a.batches for x in v[:4])
        print(f"{name:28s} {ms:8.3f} ms/batch {cnt:5.0f} launches  {fl / ms / 1e9 if ms else 0:7.1f} TF/s  "
              f"{by / ms / 1e6 if ms else 0:7.1f} GB/s")


if __name__ == "__main__":
    main()
