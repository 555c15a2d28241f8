"""Per-GPU train / eval images/sec for the other BASELINE.json configs on one MI355X (the
headline is bench.py's): config 4 = CoOp ViT-L/14 bf16 (n_ctx 16, 1000 classes, batch 32),
config 5 = CoCoOp ViT-L/14@336px bf16 (n_ctx 4, 1000 classes, 8 images per step). Synthetic
data and random-init weights of those architectures; the 8-GPU DDP forms of these configs
scale as the headline's (CoOp: class-sharded text encoding, CoCoOp: image data parallel).

    python tools/config_bench.py [--steps 5] [--warmup 2]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--eval-images", type=int, default=500)
    a = ap.parse_args()
    import torch
    import bench
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    rows = []
    for name, arch, kind, batch in [("config 4: CoOp ViT-L/14 bf16, n_ctx 16, 1000 classes", "ViT-L/14", "coop", 32),
                                    ("config 5: CoCoOp ViT-L/14@336px bf16, n_ctx 4, 1000 classes", "ViT-L/14@336px",
                                     "cocoop", 8)]:
        args = argparse.Namespace(arch=arch, classes=1000)
        build = bench.build_coop_trainer if kind == "coop" else bench.build_trainer
        tr, dm = build(args, "bf16", batch, dev, 0, n_test=a.eval_images)
        t, _ = bench.time_train(tr, dm, a.steps, a.warmup)
        e, n = bench.time_eval(tr, dm, a.eval_images)
        rows.append({"config": name, "images_per_gpu_per_step": batch,
                     "train_images_per_sec": round(batch * a.steps / t, 2), "ms_per_step": round(1e3 * t / a.steps, 2),
                     "eval_images_per_sec": round(e, 2), "eval_images": n, "dtype": "bf16",
                     "text_layout": "shared-prefix packed" if tr.model.prompt_learner.layout.pack is not None else "plain"})
        print(json.dumps(rows[-1]), flush=True)
        del tr, dm
        torch.cuda.empty_cache()
    return 0


if __name__ == "__main__":
    sys.exit(main())
