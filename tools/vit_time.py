"""Image-encoder forward alone (no text encoder beside it): ms per call at each PREC, per-site
table of one call. python tools/vit_time.py [--arch ViT-B/16] [--batch 8] [--precs fp16,fp32s,fp32]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arch", default="ViT-B/16")
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--precs", default="fp16,fp32s,fp32")
    a = ap.parse_args()
    import torch
    from fsp_amd import _native as N
    from fsp_amd.clip import synth
    from fsp_amd.clip.model import build_model
    dev = torch.device("cuda", 0)
    sd = synth.make_state_dict(a.arch, seed=0)
    arch = synth.ARCHS[a.arch]
    img = torch.from_numpy(synth.make_images(a.batch, arch.image_resolution, seed=1)).to(dev)
    for prec in a.precs.split(","):
        clip = build_model(sd, prec=prec, device=dev, text_grad=False)
        with torch.no_grad():
            for _ in range(3):
                clip.visual(img)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                clip.visual(img)
            e1.record()
            torch.cuda.synchronize()
            lib = N.load()
            lib.clipk_prof_sites_enable(1)
            clip.visual(img)
            torch.cuda.synchronize()
            sites = N.prof_sites_read()
            lib.clipk_prof_sites_enable(0)
        print(f"{a.arch} B={a.batch} {prec}: {e0.elapsed_time(e1) / 20:.3f} ms/forward", flush=True)
        for k, v in sorted(sites.items(), key=lambda kv: -kv[1][0]):
            print(f"   {k:20s} {v[0]:7.3f} ms {v[1]:3d} launches {v[2] / v[0] / 1e9 if v[0] else 0:7.1f} TF/s")
        del clip
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
