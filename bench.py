#!/usr/bin/env python3
"""Headline benchmark: CoCoOp ViT-B/16 16-shot train-step images/sec (+ eval images/sec)
on the MI355X-native path (BASELINE.json metric, configs[2]).

    python bench.py --gpus N --steps K --warmup W
    (N>1: python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N ...)

A step = one CoCoOp.forward_backward on a resident synthetic batch: ViT-B/16 image
encode -> Meta-Net -> B*C conditional prompts -> text encoder fwd + input-grad bwd ->
cosine logits -> CE -> RCCL all-reduce of the prompt grads (N>1) -> fused SGD step ->
loss.item(). Weak scaling: every rank processes its own B images (value = total images
over all ranks / max-over-ranks time). Weights are the seeded synthetic CLIP (no network).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "CoCoOp ViT-B/16 16-shot train-step images/sec at 1/2/4/8 GPUs; eval images/sec"
PEAK = {"fp16": 2500.0, "bf16": 2500.0, "amp": 2500.0, "fp32": 157.3}  # dense TFLOP/s (MI355X guide)
HBM_PEAK_GBS = 8000.0  # HBM3E, MI355X_MICROARCH.md


def flops(arch, n_cls, L):
    """SURVEY §8(d) algorithmic FLOPs (L = L_eff, the canonical text length)."""
    D, Li, p, E = arch.vision_width, arch.image_tokens, arch.vision_patch_size, arch.embed_dim
    W, tl = arch.transformer_width, arch.transformer_layers
    f_img = arch.vision_layers * (24 * Li * D * D + 4 * Li * Li * D) + 2 * (Li - 1) * D * 3 * p * p + 2 * D * E
    f_txt = tl * (24 * L * W * W + 4 * L * L * W) + 2 * W * E
    b_txt = tl * (24 * L * W * W + 8 * L * L * W)
    return f_img, f_txt, b_txt


ROOF_KERNEL = "gemm_nt_kernelIDF16_DF16_DF16_Li3ELi256ELi256"  # EPI_DQGELU fp16 persistent 256x256
PMC_FILE = os.path.join(ROOT, "profiles", "r01_pmc", "traffic.json")


def pmc_traffic(kernel_key):
    """HBM bytes per launch of the roofline kernel from the committed PMC passes of this
    workload (tools/pmc_bench.sh: separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE runs of
    bench.py; FETCH_SIZE doubled per the gfx950 note, MI355X_MICROARCH.md HBM). None if absent."""
    try:
        with open(PMC_FILE) as f:
            d = json.load(f)
    except OSError:
        return None
    hits = [v["hbm_bytes"] for k, v in d.items() if kernel_key in k]
    return hits[0] if hits else None


def cpu_baseline(arch_name, n_ctx_init, n_cls_full, sample_cls, threads):
    """Time the CPU oracle (fp32 restatement of the reference, 77-token prompts) on a
    bounded sample: 1 image x sample_cls classes, fwd + bwd; scale text cost to n_cls_full."""
    import numpy as np
    import torch
    from oracle import clip_oracle as O
    from fsp_amd.clip import synth
    from fsp_amd.clip.tokenizer import tokenize
    torch.set_num_threads(threads)
    a = synth.ARCHS[arch_name]
    sd = O.as_torch_sd(synth.make_state_dict(arch_name, seed=0))
    mp = {k: torch.from_numpy(v).requires_grad_(True)
          for k, v in synth.make_meta_net(a.embed_dim, a.transformer_width, seed=4).items()}
    names = synth.synthetic_classnames(sample_cls)
    tok = torch.from_numpy(tokenize([n_ctx_init + " " + n + "." for n in names]))
    emb = O.token_embed(sd, tok)
    n_ctx = len(n_ctx_init.split())
    ctx = emb[0, 1:1 + n_ctx].clone().requires_grad_(True)
    img = torch.from_numpy(synth.make_images(1, a.image_resolution, seed=1))
    y = torch.zeros(1, dtype=torch.long)
    with torch.no_grad():
        t0 = time.perf_counter()
        O.encode_image(sd, img)
        t_img = time.perf_counter() - t0
    t0 = time.perf_counter()
    logits = O.cocoop_logits(sd, mp, img, ctx, emb[:, :1], emb[:, 1 + n_ctx:], tok)
    loss = torch.nn.functional.cross_entropy(logits, y)
    loss.backward()
    t_all = time.perf_counter() - t0
    t_text = max(t_all - t_img, 1e-9)
    per_img = t_img + t_text * (n_cls_full / sample_cls)
    return {"value": round(1.0 / per_img, 6), "unit": "images/sec", "cores": threads, "kind": "port",
            "sample": f"oracle/clip_oracle.py fp32 CPU, CoCoOp {arch_name} 1 image x {sample_cls} classes "
                      f"fwd+bwd at 77 tokens ({t_all:.2f}s), text cost scaled linearly to {n_cls_full} classes"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=8, help="images per GPU per step")
    ap.add_argument("--classes", type=int, default=1000)
    ap.add_argument("--arch", default="ViT-B/16")
    ap.add_argument("--prec", default="fp16")
    ap.add_argument("--eval-images", type=int, default=200)
    ap.add_argument("--cpu-classes", type=int, default=50)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-prof", action="store_true")
    args = ap.parse_args()

    import torch
    from fsp_amd import dist, _native as N
    from fsp_amd.engine.config import get_cfg_default
    from fsp_amd.data.synthetic import SyntheticDataManager
    from fsp_amd.trainers.cocoop import CoCoOp
    from fsp_amd.clip import synth

    local = dist.init_from_env()
    world = dist.world_size()
    rank = dist.rank()
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    arch = synth.ARCHS[args.arch]
    cfg = get_cfg_default()
    cfg.TRAINER.NAME = "CoCoOp"
    cfg.MODEL.BACKBONE.NAME = args.arch
    cfg.INPUT.SIZE = (arch.image_resolution, arch.image_resolution)
    cfg.TRAINER.COCOOP.N_CTX = 4
    cfg.TRAINER.COCOOP.CTX_INIT = "a photo of a"
    cfg.TRAINER.COCOOP.PREC = args.prec
    cfg.DATALOADER.TRAIN_X.BATCH_SIZE = args.batch
    cfg.DATASET.NUM_SHOTS = 16
    cfg.OPTIM.MAX_EPOCH = 10
    cfg.OPTIM.WARMUP_EPOCH = 1
    cfg.OPTIM.WARMUP_TYPE = "constant"
    cfg.TEST.NO_TEST = True
    dm = SyntheticDataManager(args.classes, arch.image_resolution, args.batch, n_batches=2,
                              test_batch=100, n_test=args.eval_images, device=dev, rank=rank)
    import contextlib, io
    with contextlib.redirect_stdout(io.StringIO()):
        trainer = CoCoOp(cfg, dm=dm)
    dist.broadcast_params([p for p in trainer.model.prompt_learner.parameters()])
    trainer.num_batches = 10 ** 9  # keep update_lr out of the timed loop (epoch boundary)
    lay = trainer.model.prompt_learner.layout
    L = lay.L
    batches = dm.train_loader_x

    def step(i):
        trainer.batch_idx = i
        return trainer.forward_backward(batches[i % len(batches)])

    for i in range(args.warmup):
        step(i)
    torch.cuda.synchronize()
    dist.barrier()
    lib = N.load()
    prof = not args.no_prof
    if prof:
        lib.clipk_prof_enable(N.PROF_GEMM_DGELU)
    torch.cuda.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(i)
    torch.cuda.synchronize()
    dist.barrier()
    t = time.perf_counter() - t0
    roof = None
    if prof:
        import ctypes
        tot, cnt, work = ctypes.c_double(), ctypes.c_long(), ctypes.c_double()
        N.check(lib.clipk_prof_read(ctypes.byref(tot), ctypes.byref(cnt), ctypes.byref(work)), "prof_read")
        lib.clipk_prof_enable(N.PROF_NONE)
        if cnt.value:
            avg_ms = tot.value / cnt.value
            fl = work.value / cnt.value
            ach = fl / (avg_ms * 1e-3) / 1e12
            peak = PEAK[args.prec]  # dgelu GEMM operands: the gradient dtype (fp16 under PREC fp16)
            traffic = pmc_traffic(ROOF_KERNEL) if (args.arch, args.classes, args.batch, args.prec) == \
                ("ViT-B/16", 1000, 8, "fp16") else None
            # algorithmic bytes per launch: A [M,W] + aux h [M,4W] read, out [M,4W] written (16-bit),
            # weight [4W,W] read once
            rows = args.batch * (lay.rows_per_group if lay.pack is not None else args.classes * L)
            W = arch.transformer_width
            esz = 4 if args.prec == "fp32" else 2
            abytes = esz * (rows * (W + 4 * W * 2) + 4 * W * W)
            # the binding roofline: the longer of FLOPs at the MFMA peak and bytes at the HBM peak
            hbm_bound = abytes / (HBM_PEAK_GBS * 1e9) > fl / (peak * 1e12)
            if hbm_bound:
                achb = abytes / (avg_ms * 1e-3) / 1e9
                roof = {"bound": "hbm", "achieved": round(achb, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(achb / HBM_PEAK_GBS, 4)}
            else:
                roof = {"bound": "mfma", "achieved": round(ach, 2), "peak": peak, "unit": "TFLOP/s",
                        "frac": round(ach / peak, 4)}
            roof.update({"traffic": traffic, "algorithmic_bytes": abytes, "mfma_tflops": round(ach, 2),
                    "mfma_frac": round(ach / peak, 4),
                    "traffic_note": "traffic = HBM bytes/launch, rocprofv3 FETCH_SIZE x2 + WRITE_SIZE "
                                    "(profiles/r01_pmc)",
                    "kernel": "gemm_nt_kernel<f16,f16,f16,EPI_DQGELU> (text c_proj input-grad GEMM fused with "
                              "QuickGELU'(h), M=text rows, N=4W, K=W)",
                    "avg_launch_ms": round(avg_ms, 4), "launches": cnt.value,
                    "flops_per_launch": fl})
    tmax = dist.max_over_ranks(t)

    # eval images/sec (forward only, reference test batch 100)
    trainer.set_model_mode("eval")
    with torch.no_grad():
        for b in dm.test_loader[:1]:
            trainer.model_inference(b["img"])
        torch.cuda.synchronize()
        dist.barrier()
        te0 = time.perf_counter()
        n_eval = 0
        for b in dm.test_loader:
            trainer.model_inference(b["img"])
            n_eval += b["img"].shape[0]
        torch.cuda.synchronize()
        dist.barrier()
        te = dist.max_over_ranks(time.perf_counter() - te0)
    eval_ips = dist.sum_over_ranks(n_eval) / te if n_eval else None

    f_img, f_txt, b_txt = flops(arch, args.classes, L)
    step_flops = args.batch * (f_img + args.classes * (f_txt + b_txt))
    value = world * args.batch * args.steps / tmax
    out = {
        "metric": METRIC, "value": round(value, 3), "unit": "images/sec", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(1000 * tmax / args.steps, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": args.prec,
        "data": "synthetic (seeded U[0,1) CLIP-normalised images, random-init CLIP weights)",
        "config": {"workload": f"CoCoOp {args.arch} n_ctx=4 ctx_init='a photo of a', {args.classes} classes, "
                               f"{args.batch} images/GPU/step, train step fwd+bwd+SGD",
                   "model": f"CLIP {args.arch}", "global_batch": world * args.batch, "classes": args.classes,
                   "seq_len": L, "parallelism": f"dp{world}",
                   "text_layout": ("shared-prefix packed, %d text rows/image (plain: %d)"
                                   % (lay.rows_per_group, args.classes * L)) if lay.pack is not None
                                  else f"plain [B*C, {L}]"},
        "eval_images_per_sec": round(eval_ips, 3) if eval_ips else None,
        # reference-equivalent FLOPs (plain [B*C, L_eff] layout) per second, not executed FLOPs
        "model_tflops_per_gpu": round(step_flops * args.steps / tmax / 1e12, 2),
        "roofline": roof,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            threads = min(16, os.cpu_count() or 1)
            out["cpu_baseline"] = cpu_baseline(args.arch, "a photo of a", args.classes, args.cpu_classes, threads)
        except Exception as e:  # report, never fake
            out["cpu_baseline"] = {"value": None, "error": repr(e)}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist.is_dist():
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
