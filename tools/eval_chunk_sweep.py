"""CoCoOp eval images/sec against the text-encoder chunk size (NATIVE.MAX_TEXT_ROWS: images per
text-encoder call = MAX_TEXT_ROWS // rows per image): whether encoding fewer images per call keeps
the layer's intermediates (q|k|v, o, g = QuickGELU(h): ~1 GB per 24 images at ViT-B/16, C = 1000)
in the 256 MB Infinity Cache and runs faster per image.
    python tools/eval_chunk_sweep.py [prec]"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    prec = sys.argv[1] if len(sys.argv) > 1 else "fp16"
    from fsp_amd import dist
    dist.init_from_env()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    args = argparse.Namespace(arch="ViT-B/16", classes=1000, batch=8)
    n = 2000
    tr, dm = bench.build_trainer(args, prec, 8, dev, 0, n_test_device=n)
    rows = tr.model.prompt_learner.layout.rows_per_group
    for imgs in (100, 50, 25, 12, 8, 4, 2):
        tr.model.max_rows = imgs * rows
        bench.time_eval(tr, dm, 200)  # warm
        ips, _ = bench.time_eval(tr, dm, n)
        print(f"{prec} images per text call {imgs:4d} ({imgs * rows:7d} rows): {ips:8.1f} img/s", flush=True)


if __name__ == "__main__":
    main()
