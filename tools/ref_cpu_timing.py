"""Time the REFERENCE's own CPU path (PromptSRC CoOp / CoCoOp CustomCLIP + torch SGD,
fp32, torch CPU) for BASELINE configs 1-3, in the build container (needs /root/reference;
BASELINE.md §3, SURVEY §8(d) "CPU baseline"). Not used by bench.py (the reference does not
travel to the GPU box); the output goes to profiles/.

    python tools/ref_cpu_timing.py [--threads 8] [--classes 1000] [--configs 1 2 3]

One step = the reference forward_backward body: loss = model(image, label); zero_grad;
backward; SGD step; plus, for CoOp CE, the post-step acc re-forward (coop.py:464-469).
Median of --steps timed steps after one warm-up step. Weights: the seeded synthetic CLIP
(tests/golden/make_golden.py stand-ins; no download).
"""
from __future__ import annotations

import argparse
import json
import os
import resource
import statistics
import sys
import time

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path[:0] = [REPO, os.path.join(REPO, "tests", "golden")]

import make_golden as MG  # noqa: E402
from fsp_amd.clip import synth  # noqa: E402


def run_config(cfg_id, n_cls, steps):
    from clip.model import build_model
    a_name, trainer, batch, n_ctx, ctx_init = {
        1: ("ViT-B/32", "coop", 10, 16, ""),
        2: ("ViT-B/16", "coop", 32, 16, ""),
        3: ("ViT-B/16", "cocoop", 1, 4, "a photo of a"),
    }[cfg_id]
    if cfg_id == 1:
        n_cls = 10
    mod = __import__(f"trainers.{trainer}", fromlist=["x"])
    sd, _ = MG.build_clip(a_name)
    a = synth.ARCHS[a_name]
    clip = build_model(dict(sd), dict(MG.DESIGN, trainer="CoOp" if trainer == "coop" else "CoCoOp")).float()
    if trainer == "coop":
        cfg = MG.make_cfg(a.image_resolution, coop=dict(N_CTX=n_ctx, CTX_INIT=ctx_init, CSC=False,
                                                        CLASS_TOKEN_POSITION="end", PREC="fp32", LOSS_TYPE="ce"))
    else:
        cfg = MG.make_cfg(a.image_resolution, cocoop=dict(N_CTX=n_ctx, CTX_INIT=ctx_init, PREC="fp32",
                                                          USE_FOCAL_LOSS=False))
    model = mod.CustomCLIP(cfg, synth.synthetic_classnames(n_cls), clip)
    for n, p in model.named_parameters():
        if "prompt_learner" not in n:
            p.requires_grad_(False)
    opt = torch.optim.SGD([p for p in model.prompt_learner.parameters() if p.requires_grad], lr=0.002,
                          momentum=0.9, weight_decay=5e-4)
    img = torch.from_numpy(synth.make_images(batch, a.image_resolution, seed=1))
    lbl = torch.from_numpy(synth.make_labels(batch, n_cls, seed=2))
    model.train()

    def step():
        loss = model(img, lbl) if trainer == "cocoop" else model(img, lbl, None)
        opt.zero_grad()
        loss.backward()
        opt.step()
        loss.item()
        if trainer == "coop":  # coop.py:464-469
            with torch.no_grad():
                model(img, lbl=None, img2=None)

    times = []
    for i in range(steps + 1):
        t0 = time.perf_counter()
        step()
        if i:
            times.append(time.perf_counter() - t0)
    med = statistics.median(times)
    return {"config": cfg_id, "arch": a_name, "trainer": trainer, "classes": n_cls, "batch": batch,
            "n_ctx": n_ctx, "step_s_median": round(med, 3), "step_s_all": [round(t, 3) for t in times],
            "images_per_sec": round(batch / med, 4),
            "peak_rss_gb": round(resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 2 ** 20, 2)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--classes", type=int, default=1000)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--configs", type=int, nargs="+", default=[1, 2, 3])
    args = ap.parse_args()
    torch.set_num_threads(args.threads)
    MG._install_stubs()
    for c in args.configs:
        r = run_config(c, args.classes, args.steps)
        r.update({"threads": args.threads, "nproc": os.cpu_count(), "torch": torch.__version__})
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
