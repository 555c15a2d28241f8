#!/usr/bin/env python3
"""Headline benchmark: CoCoOp ViT-B/16 16-shot train-step images/sec (+ eval images/sec)
on the MI355X-native path (BASELINE.json metric, configs[2]), at PREC fp32s by default: the
fp32-class mode that meets the north star's 1e-3 logit bar (the reference computes in fp32,
PromptSRC/clip/model.py:699). The fp16 mode (|d logit| 0.026, outside that bar) is reported
beside it as context (``fp16``).

    python bench.py --gpus N --steps K --warmup W
    (N > 1 without a torchrun environment: this process starts
     python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 ...
     bench.py ... as a child -- before anything touches the GPU -- relays its output and exits
     with its return code; under torchrun every rank runs the benchmark and rank 0 prints)

A step = one CoCoOp.forward_backward on a resident synthetic batch: ViT-B/16 image
encode -> Meta-Net -> B*C conditional prompts -> text encoder fwd + input-grad bwd ->
cosine logits -> CE -> RCCL all-reduce of the prompt grads (N>1) -> fused SGD step.
Weak scaling: every rank processes its own B images (value = total images over all ranks /
max-over-ranks time). Weights are the seeded synthetic CLIP (no network).

The JSON line also carries (rank 0, N=1 unless noted):
* ``roofline``: the dominant kernel of the step (by time) with its algorithmic FLOPs / bytes
  per launch over its average launch time, both from hipEvents recorded around every launch
  site (clipk_prof_sites_*) during --prof-steps extra steps run right after the timed ones
  (events inside the timed region would add ~15 % wall time), and its HBM traffic from the
  committed rocprofv3 PMC passes; ``kernels``: the same for every kernel class of the step
  (GEMMs: fraction of the MFMA peak; attention / LayerNorm: GB/s and fraction of the HBM peak);
* ``eval_images_per_sec`` over --eval-images (default 50,000: SURVEY §8(d)'s full ImageNet-val
  size) distinct synthetic images resident in HBM, test batch 100, sharded over the ranks;
* ``batch1``: train images/sec at 1 image per step (the reference CoCoOp config batch size);
* ``coop``: BASELINE config 2 -- CoOp n_ctx 16, ViT-B/16, 1000 classes, batch 32: train and
  eval images/sec;
* ``batch1_class_shard`` (N > 1): the reference's CoCoOp batch of 1 image per step with its
  1,000 classes sharded over the N ranks (SURVEY §8(e) Option B: logit all-gather + SUM
  all-reduce of the prompt gradients), strong scaling of that step;
* ``config4`` / ``config5`` (N = 1): BASELINE configs 4 (CoOp ViT-L/14 bf16, 32 images/step) and 5
  (CoCoOp ViT-L/14@336px bf16, 8 images/step) per GPU, train and eval images/sec;
* ``fp16`` / ``fp32``: the headline workload at PREC fp16 (16-bit forward and gradients, the
  fastest mode, outside the 1e-3 bar) and PREC fp32 (f32-input MFMA): train over 10 steps, eval
  over 50,000 / 5,000 images, each with its own roofline;
* ``cpu_baseline``: the oracle (fp32 restatement) on the host cores, with nproc stated, and the
  reference's own CPU path at 1,000 classes as measured in the build container
  (tools/ref_cpu_timing.py -> profiles/r03_ref_cpu_timing.jsonl; the reference does not travel
  to the GPU box).
"""
from __future__ import annotations

import argparse
import contextlib
import io
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

def metric_name(arch):
    """BASELINE.json's metric, for the --arch being run (ViT-B/16 by default)."""
    return f"CoCoOp {arch} 16-shot train-step images/sec at 1/2/4/8 GPUs; eval images/sec"


REF_CPU_FILE = os.path.join(ROOT, "profiles", "r03_ref_cpu_timing.jsonl")


_T0 = time.time()


def log(msg):
    """Progress on stderr (the JSON line alone goes to stdout): a long default run keeps
    writing, so a watchdog on silent commands does not take it for hung."""
    print(f"[bench {time.time() - _T0:7.1f}s] {msg}", file=sys.stderr, flush=True)


def launcher_cmd(argv, n, port):
    """The torchrun command bench.py --gpus N (N > 1) starts as its child: one rank per GPU
    of this node, rendezvous on 127.0.0.1, the same bench arguments."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
            "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def reference_cpu(arch, classes):
    """The reference's own CPU train step (PromptSRC CoCoOp CustomCLIP + torch SGD, fp32) at
    this config, measured in the build container (8 threads): images/sec, or None."""
    try:
        with open(REF_CPU_FILE) as f:
            rows = [json.loads(l) for l in f if l.strip()]
    except OSError:
        return None
    for r in rows:
        if r.get("config") == 3 and r.get("arch") == arch and r.get("classes") == classes:
            return {"value": r["images_per_sec"], "unit": "images/sec", "cores": r["threads"], "kind": "reference",
                    "sample": (f"reference CoCoOp {arch} (PromptSRC/trainers/cocoop.py CustomCLIP + torch.optim.SGD, "
                               f"fp32, 77-token prompts), 1 image x {classes} classes per step, median of "
                               f"{len(r['step_s_all'])} steps ({r['step_s_median']} s/step), {r['threads']} threads "
                               f"of the build container's {r['nproc']}-core Xeon (not the GPU box: the reference "
                               f"does not travel); {REF_CPU_FILE[len(ROOT) + 1:]}")}
    return None
# dense TFLOP/s (MI355X guide); fp32s: the fp16 MFMA peak / 3 (3 fp16 MFMAs per fp32-class product,
# include/clipk.h CLIPK_F32S), the ceiling for its algorithmic (fp32) FLOPs
PEAK = {"fp16": 2500.0, "bf16": 2500.0, "amp": 2500.0, "fp32": 157.3, "fp32s": 2500.0 / 3,
        # PREC fp32s on fp16-valued weights (split mode 2, CLIPK_F32S16): 2 MFMAs per product
        # (the LayerNorm-folded qkv / c_fc forward keep 3: their fraction is understated here)
        "fp32s16": 2500.0 / 2}
HBM_PEAK_GBS = 8000.0  # HBM3E, MI355X_MICROARCH.md
# batch-1 lines: ~2.7 ms steps, so 50 timed steps (10 let one host hiccup move the mean ~20 %:
# 3.32 ms in one round-4 run against 2.70 over 50 steps of tools/b1_time.py on the same build)
B1_STEPS = 50
# the latest round's PMC passes (tools/pmc_bench.sh), else the previous round's
PMC_FILES = {  # per PREC: the latest round's PMC passes of that workload (tools/pmc_bench.sh)
    "fp32s": os.path.join(ROOT, "profiles", "r06_pmc", "traffic.json"),
    "fp16": next((f for f in (os.path.join(ROOT, "profiles", r, "traffic.json") for r in ("r06_pmc_fp16", "r05_pmc"))
                  if os.path.exists(f)), os.path.join(ROOT, "profiles", "r05_pmc", "traffic.json")),
}

# kernel classes of the step: launch sites that run the same kernel instantiation (rocprofv3
# kernel-name key, for the PMC traffic lookup) -- the text GEMMs by role, attention, LN. Each
# class's bound is decided from its own algorithmic FLOPs and bytes per launch (kernel_table).
DX_SITES = ["text.fc_dx", "text.qkv_dx", "text.out_dx", "text.fc_dx_eot", "text.out_dx_eot"]
KERNELS = {
    "gemm_dx_n512": (DX_SITES, "EPI_NONE 192x256"),
    "gemm_proj_fwd": (["text.proj_fwd"], "EPI_BIAS_RES N=512 K=2048"),
    "gemm_dgelu": (["text.proj_dx_dgelu", "text.proj_dx_dgelu_eot"],
                   "EPI_DQGELU | QGELU_DERIV (acc x the saved quickgelu')"),
    "gemm_fc_fwd": (["text.fc_fwd"], "EPI_BIAS_QGELU | QGELU_DERIV N=2048 (QuickGELU(h) and quickgelu'(h); ln_2 folded)"),
    "gemm_qkv_fwd": (["text.qkv_fwd"], "EPI_BIAS N=1536 (ln_1 folded)"),
    "gemm_out_fwd": (["text.out_fwd"], "EPI_BIAS_RES N=512"),
    "attn_bwd": (["text.attn_bwd"], "attn_prefix_bwd_lds"),
    "attn_fwd": (["text.attn_fwd"], "attn_prefix_fwd_lds"),
    "ln_bwd": (["text.ln_bwd"], "ln_bwd_kernel"),
    "ln_fwd": (["text.ln_fwd"], "ln_fwd_kernel"),
    "ln_stats": (["text.ln_stats"], "ln_stats_merge_kernel (LN fold statistics)"),
    "vit": (["vit.patch_embed", "vit.qkv_fwd", "vit.attn_fwd", "vit.out_fwd", "vit.fc_fwd", "vit.proj_fwd",
             "vit.ln_fwd", "vit.ln_stats", "vit.eot_gather", "vit.head"], "ViT forward (all sites)"),
}
# the dominant class split by GEMM shape (M rows x N 512 x K): the 11 full-row launches of each
# input-grad GEMM, and the last layer's compact EOT-row launches (M = B*C)
DX_SHAPES = {"fc_dx K=2048": ["text.fc_dx"], "qkv_dx K=1536": ["text.qkv_dx"], "out_dx K=512": ["text.out_dx"],
             "eot fc_dx+out_dx": ["text.fc_dx_eot", "text.out_dx_eot"]}
# rocprofv3 kernel-name keys of a class, per PREC (a class may run several instantiations: fp32s's
# fc_dx reads its A pre-split, qkv_dx / out_dx do not)
# (rocprofv3 writes the kernel names mangled or demangled depending on its build: each class lists
# both forms)
ROOF_PMC_KEY = {
    "fp16": {"gemm_dx_n512": ("gemm_nt_kernelIDF16_DF16_fLi4ELi192ELi256",
                              "gemm_nt_kernel<_Float16, _Float16, float, 4, 192, 256,"),
             "gemm_dgelu": ("gemm_nt_kernelIDF16_DF16_DF16_Li6E", "gemm_nt_kernel<_Float16, _Float16, _Float16, 6,"),
             "gemm_proj_fwd": ("gemm_nt_kernelIDF16_DF16_DF16_Li1ELi192ELi256ELi2ELi4ELb1ELi128ELi2ELb0ELb1E",
                               "gemm_nt_kernel<_Float16, _Float16, _Float16, 1, 192, 256, 2, 4, true, 128, 2, false, true,"),
             "attn_bwd": ("attn_prefix_bwd_lds",)},
    "fp32s": {"gemm_dx_n512": ("gemm_nt_kernelINS_4f32hEffLi4ELi192ELi256ELi2ELi4ELb1E",
                               "gemm_nt_kernel<clipk::f32h, float, float, 4, 192, 256, 2, 4, true,"),
              "gemm_dgelu": ("gemm_nt_kernelINS_4f32hEffLi6ELi192ELi256ELi2ELi4ELb1E",
                             "gemm_nt_kernel<clipk::f32h, float, float, 6, 192, 256, 2, 4, true,"),
              "gemm_proj_fwd": ("gemm_nt_kernelINS_4f32hEffLi1ELi192ELi256ELi2ELi4ELb1E",
                                "gemm_nt_kernel<clipk::f32h, float, float, 1, 192, 256, 2, 4, true,"),
              "gemm_fc_fwd": ("gemm_nt_kernelINS_4f32hEffLi5ELi192ELi256ELi2ELi4ELb1E",
                              "gemm_nt_kernel<clipk::f32h, float, float, 5, 192, 256, 2, 4, true,"),
              "attn_bwd": ("attn_prefix_bwd_f32",)},
}


def flops(arch, n_cls, L):
    """SURVEY §8(d) algorithmic FLOPs (L = L_eff, the canonical text length)."""
    D, Li, p, E = arch.vision_width, arch.image_tokens, arch.vision_patch_size, arch.embed_dim
    W, tl = arch.transformer_width, arch.transformer_layers
    f_img = arch.vision_layers * (24 * Li * D * D + 4 * Li * Li * D) + 2 * (Li - 1) * D * 3 * p * p + 2 * D * E
    f_txt = tl * (24 * L * W * W + 4 * L * L * W) + 2 * W * E
    b_txt = tl * (24 * L * W * W + 8 * L * L * W)
    return f_img, f_txt, b_txt


def pmc_traffic(kernel_key, prec="fp32s"):
    """HBM bytes per launch of a kernel class from the committed PMC passes of this workload
    (tools/pmc_bench.sh: separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE runs of bench.py at that
    PREC; FETCH_SIZE doubled per the gfx950 note, MI355X_MICROARCH.md HBM): the launch-weighted
    mean over the kernels whose name holds the key (a string, or a tuple of alternative forms).
    None if absent."""
    try:
        with open(PMC_FILES[prec]) as f:
            d = json.load(f)
    except (OSError, KeyError):
        return None
    keys = (kernel_key,) if isinstance(kernel_key, str) else tuple(kernel_key or ())
    hits = [(v["hbm_bytes"], v.get("launches", 1)) for k, v in d.items() if any(x and x in k for x in keys)]
    n = sum(c for _, c in hits)
    return round(sum(b * c for b, c in hits) / n, 1) if n else None


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
        O.encode_image(sd, img)  # warm-up
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
    scaled = (f"text cost scaled linearly to {n_cls_full} classes" if sample_cls != n_cls_full
              else "the full class set, unscaled")
    return {"value": round(1.0 / per_img, 6), "unit": "images/sec", "cores": threads, "kind": "port",
            "nproc": os.cpu_count(),
            "sample": f"oracle fp32 CPU, CoCoOp {arch_name} 1 image x {sample_cls} classes fwd+bwd at 77 tokens "
                      f"({t_all:.1f}s) on {threads} threads (nproc {os.cpu_count()}), {scaled}"}


def kernel_table(sites, steps, prec):
    """Per kernel class: launches, avg ms, algorithmic TF/s and GB/s per launch, fractions."""
    peak = PEAK[prec]
    out = {}
    for name, (members, desc) in KERNELS.items():
        ms = sum(sites[s][0] for s in members if s in sites)
        n = sum(sites[s][1] for s in members if s in sites)
        fl = sum(sites[s][2] for s in members if s in sites)
        by = sum(sites[s][3] for s in members if s in sites)
        if not n:
            continue
        sec = ms * 1e-3
        tf = fl / sec / 1e12 if fl else 0.0
        gbs = by / sec / 1e9
        # the binding roofline of this class: the longer of its FLOPs at the MFMA peak and its
        # bytes at the HBM peak (arithmetic intensity vs the ridge point peak / 8 TB/s)
        bound = "hbm" if (fl == 0 or by / (HBM_PEAK_GBS * 1e9) > fl / (peak * 1e12)) else "mfma"
        out[name] = {"kernel": desc, "launches_per_step": round(n / steps, 2), "ms_per_step": round(ms / steps, 4),
                     "avg_launch_ms": round(ms / n, 4), "tflops": round(tf, 1), "mfma_frac": round(tf / peak, 4),
                     "gbs": round(gbs, 1), "hbm_frac": round(gbs / HBM_PEAK_GBS, 4), "bound": bound,
                     "roof_frac": round(gbs / HBM_PEAK_GBS if bound == "hbm" else tf / peak, 4),
                     "flop_per_byte": round(fl / by, 1) if by else None,
                     "flops_per_launch": fl / n, "bytes_per_launch": by / n}
    return out


def dx_by_shape(sites, steps, prec):
    """The N = 512 input-grad class per GEMM shape: launches per step, avg us per launch, TF/s and
    the fraction of the MFMA peak (names the worst shape of the roofline kernel)."""
    out = {}
    for name, members in DX_SHAPES.items():
        ms = sum(sites[x][0] for x in members if x in sites)
        n = sum(sites[x][1] for x in members if x in sites)
        fl = sum(sites[x][2] for x in members if x in sites)
        if n:
            tf = fl / (ms * 1e-3) / 1e12
            out[name] = {"launches": round(n / steps, 1), "avg_us": round(1000 * ms / n, 1), "tflops": round(tf, 1),
                         "mfma_frac": round(tf / PEAK[prec], 4)}
    return out


def executed_gemm_tflops(sites, steps, step_s):
    """GEMM FLOPs the step actually launches (every text + ViT GEMM site: shared-prefix packed
    rows, EOT-only last layer) per second of step time."""
    fl = sum(v[2] for v in sites.values()) / steps
    return round(fl / step_s / 1e12, 2)


def roofline_of(table, prec):
    name = max((k for k in table if k != "vit"), key=lambda k: table[k]["ms_per_step"])
    k = table[name]
    peak = PEAK[prec]
    fl, by, avg = k["flops_per_launch"], k["bytes_per_launch"], k["avg_launch_ms"] * 1e-3
    # the binding roofline: the longer of FLOPs at the MFMA peak and bytes at the HBM peak
    hbm_bound = fl == 0 or by / (HBM_PEAK_GBS * 1e9) > fl / (peak * 1e12)
    if hbm_bound:
        ach = by / avg / 1e9
        r = {"bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
             "frac": round(ach / HBM_PEAK_GBS, 4)}
    else:
        ach = fl / avg / 1e12
        r = {"bound": "mfma", "achieved": round(ach, 2), "peak": peak, "unit": "TFLOP/s", "frac": round(ach / peak, 4)}
    base = "fp32s" if prec.startswith("fp32s") else prec
    key = ROOF_PMC_KEY.get(base, {}).get(name)
    r.update({"traffic": pmc_traffic(key, base) if key else None,
              "kernel_class": name, "kernel": k["kernel"], "avg_launch_ms": k["avg_launch_ms"],
              "flops_per_launch": fl, "algorithmic_bytes": by})
    if key and base in PMC_FILES:
        r["traffic_note"] = ("HBM bytes/launch, rocprofv3 FETCH_SIZE x2 + WRITE_SIZE, launch-weighted over the class's "
                             "kernels (" + os.path.relpath(os.path.dirname(PMC_FILES[base]), ROOT) + ")")
    return r


def build_coop_trainer(args, prec, batch, dev, rank, n_test=0, n_test_device=0):
    """BASELINE config 2: CoOp n_ctx=16 (random init, class token at the end, shared context),
    ViT-B/16, fp16, 1000 classes (ImageNet-LT size), train batch 32 (configs/trainers/CoOp/
    vit_b16.yaml:3), test batch 100."""
    from fsp_amd.engine.config import get_cfg_default
    from fsp_amd.data.synthetic import SyntheticDataManager
    from fsp_amd.trainers.coop import CoOp
    from fsp_amd.clip import synth
    arch = synth.ARCHS[args.arch]
    cfg = get_cfg_default()
    cfg.TRAINER.NAME = "CoOp"
    cfg.MODEL.BACKBONE.NAME = args.arch
    cfg.INPUT.SIZE = (arch.image_resolution, arch.image_resolution)
    c = cfg.TRAINER.COOP
    c.N_CTX, c.CTX_INIT, c.CSC, c.CLASS_TOKEN_POSITION, c.PREC = 16, "", False, "end", prec
    cfg.DATALOADER.TRAIN_X.BATCH_SIZE = batch
    cfg.DATASET.NUM_SHOTS = 16
    cfg.OPTIM.MAX_EPOCH = 10
    cfg.TEST.NO_TEST = True
    cfg.MODEL.SYNTH_FP16 = getattr(args, "weights", "fp16") == "fp16"
    dm = SyntheticDataManager(args.classes, arch.image_resolution, batch, n_batches=2, test_batch=100,
                              n_test=n_test, device=dev, rank=rank, n_test_device=n_test_device)
    with contextlib.redirect_stdout(io.StringIO()):
        trainer = CoOp(cfg, dm=dm)
    trainer.num_batches = 10 ** 9
    return trainer, dm


def build_trainer(args, prec, batch, dev, rank, n_test=0, n_test_device=0, class_shard=False):
    from fsp_amd.engine.config import get_cfg_default
    from fsp_amd.data.synthetic import SyntheticDataManager
    from fsp_amd.trainers.cocoop import CoCoOp
    from fsp_amd.clip import synth
    arch = synth.ARCHS[args.arch]
    cfg = get_cfg_default()
    cfg.TRAINER.NAME = "CoCoOp"
    cfg.MODEL.BACKBONE.NAME = args.arch
    cfg.INPUT.SIZE = (arch.image_resolution, arch.image_resolution)
    cfg.TRAINER.COCOOP.N_CTX = 4
    cfg.TRAINER.COCOOP.CTX_INIT = "a photo of a"
    cfg.TRAINER.COCOOP.PREC = prec
    cfg.DATALOADER.TRAIN_X.BATCH_SIZE = batch
    cfg.DATASET.NUM_SHOTS = 16
    cfg.OPTIM.MAX_EPOCH = 10
    cfg.OPTIM.WARMUP_EPOCH = 1
    cfg.OPTIM.WARMUP_TYPE = "constant"
    cfg.TEST.NO_TEST = True
    cfg.NATIVE.COCOOP_SHARD = "class" if class_shard else "image"
    cfg.MODEL.SYNTH_FP16 = getattr(args, "weights", "fp16") == "fp16"
    dm = SyntheticDataManager(args.classes, arch.image_resolution, batch, n_batches=2, test_batch=100,
                              n_test=n_test, device=dev, rank=rank, n_test_device=n_test_device)
    with contextlib.redirect_stdout(io.StringIO()):
        trainer = CoCoOp(cfg, dm=dm)  # broadcasts the prompt parameters (N>1)
    trainer.num_batches = 10 ** 9  # keep update_lr out of the timed loop (epoch boundary)
    return trainer, dm


def time_train(trainer, dm, steps, warmup, batch=None, prof_steps=0):
    """Warm-up, then `steps` timed steps (barrier + synchronize both sides, max over ranks);
    then, when prof_steps > 0, that many more steps with hipEvents around every launch
    site (kept out of the timed region: ~300 event records per step add ~15 % wall time),
    returning the per-site table."""
    import torch
    from fsp_amd import dist, _native as N
    batches = dm.train_loader_x
    if batch is not None:
        batches = [{"img": b["img"][:batch], "label": b["label"][:batch]} for b in batches]

    def step(i):
        trainer.batch_idx = i
        trainer.next_batch = batches[(i + 1) % len(batches)]  # as TrainerX.run_epoch's lookahead
        return trainer.forward_backward(batches[i % len(batches)])

    for i in range(warmup):
        step(i)
    torch.cuda.synchronize()
    dist.barrier()
    t0 = time.perf_counter()
    for i in range(steps):
        step(i)
    torch.cuda.synchronize()
    dist.barrier()
    t = time.perf_counter() - t0
    table = None
    if prof_steps > 0:
        lib = N.load()
        lib.clipk_prof_sites_enable(1)
        for i in range(prof_steps):
            step(i)
        torch.cuda.synchronize()
        table = N.prof_sites_read()
        lib.clipk_prof_sites_enable(0)
    return dist.max_over_ranks(t), table


def time_eval(trainer, dm, n_images):
    """Forward-only images/sec over n_images (test batch 100; the resident synthetic test
    batches are cycled)."""
    import torch
    from fsp_amd import dist
    if n_images <= 0:  # profiling runs of the train step alone
        return 0.0, 0
    trainer.set_model_mode("eval")
    tl = dm.test_loader
    nb = (n_images + 99) // 100
    hint = hasattr(trainer.model, "prefetch_image_features")  # as TrainerX.test's lookahead
    with torch.no_grad():
        trainer.model_inference(tl[0]["img"])
        torch.cuda.synchronize()
        dist.barrier()
        t0 = time.perf_counter()
        n = 0
        for i in range(nb):
            x = tl[i % len(tl)]["img"]
            if hint:
                trainer.model.next_image = tl[(i + 1) % len(tl)]["img"] if i + 1 < nb else None
            trainer.model_inference(x)
            n += x.shape[0]
        torch.cuda.synchronize()
        dist.barrier()
        te = dist.max_over_ranks(time.perf_counter() - t0)
    trainer.set_model_mode("train")
    return dist.sum_over_ranks(n) / te, n


def time_grad_allreduce(params, iters=50, warmup=10):
    """The step's gradient all-reduce alone (dist.allreduce_grads over the prompt learner's
    trainable parameters: one flat fp32 bucket, RCCL over xGMI at N > 1), barrier + sync around
    `iters` calls, max over ranks. Run after the timed region; it sums into the grads."""
    import torch
    from fsp_amd import dist
    ps = [p for p in params if p.requires_grad]
    for p in ps:
        if p.grad is None:
            p.grad = torch.zeros_like(p)
    cuda = ps[0].is_cuda

    def sync():
        if cuda:
            torch.cuda.synchronize()
        dist.barrier()

    for _ in range(warmup):
        dist.allreduce_grads(ps, average=False)
    sync()
    t0 = time.perf_counter()
    for _ in range(iters):
        dist.allreduce_grads(ps, average=False)
    sync()
    t = dist.max_over_ranks(time.perf_counter() - t0)
    return {"bytes": 4 * sum(p.numel() for p in ps), "us_per_call": round(1e6 * t / iters, 1), "iters": iters,
            "backend": torch.distributed.get_backend() if dist.is_dist() else None}


# |d logit| of each PREC against the reference's own golden logits at the headline shape
# (tests/test_parity_gpu.py test_headline_batch8_vs_golden, tests/golden/cocoop_vitb16_c1000_b8.npz)
# (fp32s on the benched fp16-valued weights: test_headline_batch8_w16_vs_golden, cocoop_vitb16_c1000_b8_w16.npz;
# profiles/r06h/t_headline_reports.txt)
LOGIT_ERR = {"fp32s": "2.3e-5 (fp16-valued weights, as benched; 2.7e-5 on fp32-valued ones)", "fp32": "2.9e-5",
             "fp16": "0.024 (outside the north star's 1e-3)"}


def peak_key(prec, trainer):
    """The PEAK entry a PREC's GEMM FLOPs are priced against: fp32s on fp16-valued weights (split
    mode 2, CLIPK_F32S16) forms 2 fp16 MFMAs per product, else 3."""
    if prec == "fp32s" and trainer.model.text_core.split_mode == 2:
        return "fp32s16"
    return prec


def precision_line(args, prec, dev, rank, world, steps=10, warmup=2, n_eval=5000, prof=True):
    """The headline workload at another PREC: train img/s over `steps` timed steps, eval img/s
    over n_eval distinct resident images, and the roofline of its dominant kernel class
    (site events in 2 extra steps)."""
    import torch
    from fsp_amd import dist
    from fsp_amd.clip.model import TextEncoderCore
    tr, dm = build_trainer(args, prec, args.batch, dev, rank, n_test_device=n_eval)
    retries0 = TextEncoderCore.split_retries
    t, sites = time_train(tr, dm, steps, warmup, prof_steps=2 if prof else 0)
    retries = TextEncoderCore.split_retries - retries0
    # the MFMA peak the dominant class is priced against: 3 or 2 fp16 MFMAs per product
    pk = peak_key(prec, tr)
    table = kernel_table(sites, 2, pk) if sites else None
    e, n = time_eval(tr, dm, n_eval)
    roof = roofline_of(table, pk) if table else None
    if roof:  # the bench line carries the headline's full roofline record; here the essentials
        roof = {k: roof[k] for k in ("bound", "achieved", "peak", "unit", "frac", "kernel_class", "avg_launch_ms")}
    line = {"images_per_sec": round(world * args.batch * steps / t, 3), "ms_per_step": round(1000 * t / steps, 3),
            "steps": steps, "eval_images_per_sec": round(e, 3), "eval_images": int(dist.sum_over_ranks(n)),
            "logit_err_vs_reference": LOGIT_ERR.get(prec), "roofline": roof,
            # the classes over 0.5 ms/step: [ms/step, bound, fraction of that roof]
            "kernels": ({k: [v["ms_per_step"], v["bound"], v["roof_frac"]] for k, v in table.items()
                         if v["ms_per_step"] >= 0.5} if table else None)}
    if prec == "fp32s":
        line["peak_note"] = ("peak = fp16 MFMA peak / %d (%d fp16 MFMAs per fp32-class product)"
                             % ((2, 2) if pk == "fp32s16" else (3, 3)))
        # 2: fp16-valued weights, the GEMMs but the LayerNorm-folded ones skip the weight-lo
        # product (CLIPK_F32S16, bitwise the same results); 1: every GEMM 3 MFMAs per product
        line["split_mode"] = {"text": tr.model.text_core.split_mode, "vision": tr.model.image_encoder.split_mode}
        # backward passes re-run at the lower gradient scale after a range overflow (warm-up,
        # timed and profiled steps; each one doubles that step's backward)
        line["split_retries"] = retries
    del tr, dm
    torch.cuda.empty_cache()
    return line


def baseline_config_line(args, dev, rank, world, steps=10, warmup=3, n_eval=5000):
    """BASELINE.json configs 4 / 5 for --arch ViT-L/14 / ViT-L/14@336px (bf16, 1,000 classes,
    synthetic data, random-init weights of those architectures): config 4 = CoOp n_ctx 16 at 32
    images per GPU per step (class-sharded text encoding at N > 1), config 5 = CoCoOp n_ctx 4 at
    8 images per GPU per step (image data parallel). Train and eval images/sec (whole job)."""
    import torch
    from fsp_amd import dist
    if args.arch == "ViT-L/14":
        name, batch = "config 4: CoOp ViT-L/14 bf16, n_ctx 16, 1000 classes, 32 images/GPU/step", 32
        tr, dm = build_coop_trainer(args, "bf16", batch, dev, rank, n_test_device=n_eval)
    else:
        name, batch = "config 5: CoCoOp ViT-L/14@336px bf16, n_ctx 4, 1000 classes, 8 images/GPU/step", 8
        tr, dm = build_trainer(args, "bf16", batch, dev, rank, n_test_device=n_eval)
    t, _ = time_train(tr, dm, steps, warmup)
    e, n = time_eval(tr, dm, n_eval)
    line = {"workload": name, "images_per_sec": round(world * batch * steps / t, 3),
            "ms_per_step": round(1000 * t / steps, 3), "steps": steps, "eval_images_per_sec": round(e, 3),
            "eval_images": int(dist.sum_over_ranks(n)), "dtype": "bf16",
            "text_layout": "shared-prefix packed" if tr.model.prompt_learner.layout.pack is not None else "plain"}
    del tr, dm
    torch.cuda.empty_cache()
    return line


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=8, help="images per GPU per step")
    ap.add_argument("--classes", type=int, default=1000)
    ap.add_argument("--arch", default="ViT-B/16")
    ap.add_argument("--prec", default="fp32s",
                    help="headline PREC (fp32s: the fp32-class mode meeting the 1e-3 logit bar)")
    ap.add_argument("--eval-images", type=int, default=50000)
    ap.add_argument("--cpu-classes", type=int, default=0,
                    help="classes in the CPU-baseline sample (0: all of --classes, no scaling)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--prof-steps", type=int, default=3, help="steps after the timed ones with per-site hipEvents")
    ap.add_argument("--no-prof", action="store_true", help="no per-site profiling steps")
    ap.add_argument("--no-extra", action="store_true", help="skip the fp32 / batch-1 lines")
    ap.add_argument("--no-configs", action="store_true", help="skip the BASELINE config 4 / 5 lines")
    ap.add_argument("--weights", choices=("fp16", "fp32"), default="fp16",
                    help="synthetic CLIP weights rounded to fp16 (as the released checkpoints) or fp32")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # one rank per GPU: torchrun as a CHILD process (this process has not touched the GPU)
        import subprocess
        env = dict(os.environ)
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        rc = subprocess.call(launcher_cmd(sys.argv[1:], args.gpus, _free_port()), env=env)
        sys.exit(rc)

    import torch
    from fsp_amd import dist
    from fsp_amd import _native as N
    from fsp_amd.clip import synth

    local = dist.init_from_env()
    world = dist.world_size()
    rank = dist.rank()
    if world != args.gpus:
        raise SystemExit(f"bench.py --gpus {args.gpus} but the process group has {world} ranks")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    arch = synth.ARCHS[args.arch]
    n_eval_rank = dist.shard_range(args.eval_images)[1] - dist.shard_range(args.eval_images)[0]

    log(f"headline: {args.arch} B={args.batch} C={args.classes} {args.prec}")
    trainer, dm = build_trainer(args, args.prec, args.batch, dev, rank, n_test_device=n_eval_rank)
    lay = trainer.model.prompt_learner.layout
    L = lay.L
    n_prof = 0 if args.no_prof else args.prof_steps
    t, sites = time_train(trainer, dm, args.steps, args.warmup, prof_steps=n_prof)
    pk = peak_key(args.prec, trainer)
    table = kernel_table(sites, n_prof, pk) if sites else None
    roof = roofline_of(table, pk) if table else None
    log(f"headline train {1000 * t / args.steps:.3f} ms/step; eval")
    eval_ips, n_eval = time_eval(trainer, dm, n_eval_rank)
    log(f"eval {eval_ips:.1f} img/s")

    f_img, f_txt, b_txt = flops(arch, args.classes, L)
    step_flops = args.batch * (f_img + args.classes * (f_txt + b_txt))
    _, f77, b77 = flops(arch, args.classes, 77)
    step_flops_77 = args.batch * (f_img + args.classes * (f77 + b77))
    value = world * args.batch * args.steps / t
    out = {
        "metric": metric_name(args.arch), "value": round(value, 3), "unit": "images/sec", "n_gpus": world,
        "rccl_world": world, "backend": torch.distributed.get_backend() if dist.is_dist() else None,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(1000 * t / args.steps, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": args.prec,
        "dtype_note": {"fp32s": "fp32-class: fp32 activations, residual stream, LayerNorm, softmax and attention; "
                                "every GEMM product as fp16 hi / lo parts on the 16-bit MFMA (~22 significant "
                                "bits per operand, fp32 accumulate) -- the reference computes in fp32 "
                                "(PromptSRC/clip/model.py:699)",
                       "fp16": "fp16 forward and gradients (outside the 1e-3 logit bar)"}.get(args.prec, args.prec),
        "logit_err_vs_reference": LOGIT_ERR.get(args.prec),
        "data": "synthetic (seeded U[0,1) CLIP-normalised images, random-init CLIP weights%s)"
                % (" rounded to fp16, as the released CLIP checkpoints hold them" if args.weights == "fp16" else ""),
        "config": {"workload": f"CoCoOp {args.arch} n_ctx=4 ctx_init='a photo of a', {args.classes} classes, "
                               f"{args.batch} images/GPU/step, train step fwd+bwd+SGD",
                   "model": f"CLIP {args.arch}", "global_batch": world * args.batch, "classes": args.classes,
                   "seq_len": L, "parallelism": f"dp{world}",
                   "text_layout": ("shared-prefix packed, %d text rows/image (plain: %d)"
                                   % (lay.rows_per_group, args.classes * L)) if lay.pack is not None
                                  else f"plain [B*C, {L}]",
                   "vision": ("the NEXT batch's frozen ViT forward on a side stream (NATIVE.PREFETCH_VISION, "
                              "TrainerX.run_epoch's lookahead): one ViT fwd + one text fwd+bwd per step"
                              if trainer.cfg.NATIVE.get("PREFETCH_VISION", False) else "in line")},
        "eval_images_per_sec": round(eval_ips, 3),
        "eval_images": int(dist.sum_over_ranks(n_eval)),
        "eval_note": "forward only, test batch 100, distinct resident images sharded over the ranks",
        "source_digest": N.library_digest()[:16],
        # SURVEY §8(d) algorithmic FLOPs per second: the plain [B*C, L_eff] layout (L_eff = max EOT
        # + 1), the same at the reference's 77 tokens, and the GEMM FLOPs the step executes
        # (shared-prefix packed rows, EOT-only last layer; attention not counted)
        "model_tflops_per_gpu": round(step_flops * args.steps / t / 1e12, 2),
        "model_tflops_per_gpu_l77": round(step_flops_77 * args.steps / t / 1e12, 2),
        "executed_gemm_tflops_per_gpu": executed_gemm_tflops(sites, n_prof, t / args.steps) if sites else None,
        "roofline": roof,
        "dx_by_shape": dx_by_shape(sites, n_prof, pk) if sites else None,
        "peak_note": ("fp32s GEMM FLOPs priced at the fp16 MFMA peak / %d (%d fp16 MFMAs per fp32-class product)"
                      % ((2, 2) if pk == "fp32s16" else (3, 3))) if args.prec == "fp32s" else None,
        # per kernel class: [launches/step, ms/step, bound, fraction of that roof, TF/s, GB/s]
        "kernels": ({k: [v["launches_per_step"], v["ms_per_step"], v["bound"], v["roof_frac"], v["tflops"], v["gbs"]]
                     for k, v in table.items()} if table else None),
    }
    if args.prec == "fp32s":
        out["split_mode"] = {"text": trainer.model.text_core.split_mode, "vision": trainer.model.image_encoder.split_mode}
    if world > 1:  # the step's gradient all-reduce measured on its own (part of ms_per_step above)
        out["grad_allreduce"] = time_grad_allreduce(list(trainer.model.prompt_learner.parameters()))
    del trainer, dm
    torch.cuda.empty_cache()
    if not args.no_extra and world > 1:
        # the reference's CoCoOp batch (1 image / step) with the classes sharded over the ranks
        tr1, dm1 = build_trainer(args, args.prec, 1, dev, 0, class_shard=True)
        t1, _ = time_train(tr1, dm1, B1_STEPS, 5)
        out["batch1_class_shard"] = {"images_per_sec": round(B1_STEPS / t1, 3),
                                     "ms_per_step": round(1000 * t1 / B1_STEPS, 3), "steps": B1_STEPS,
                                     "global_batch": 1, "classes_per_rank": tr1.model.prompt_learner.layout.n_cls,
                                     "scaling": "strong"}
        del tr1, dm1
        torch.cuda.empty_cache()
    if not args.no_extra and world == 1:  # the N > 1 scaling runs report the headline lines only
        # the reference's batch size for CoCoOp (configs/trainers/CoCoOp/*.yaml: 1 image/step)
        for bp in dict.fromkeys((args.prec, "fp16")):  # the headline PREC, then fp16 (context)
            sfx = "" if bp == args.prec else "_" + bp
            log(f"batch1 {bp}")
            tr1, dm1 = build_trainer(args, bp, 1, dev, rank)
            t1, _ = time_train(tr1, dm1, B1_STEPS, 5)
            out["batch1" + sfx] = {"images_per_sec": round(world * B1_STEPS / t1, 3),
                                   "ms_per_step": round(1000 * t1 / B1_STEPS, 3), "steps": B1_STEPS,
                                   "images_per_gpu_per_step": 1, "dtype": bp}
            del tr1, dm1
            torch.cuda.empty_cache()
            # single-GPU proxy of batch-1 class sharding at N = 2 / 4 / 8: one rank's
            # work -- B = 1 at C / N classes -- timed alone, a lower bound on the N-GPU step (the
            # logit all-gather and the gradient all-reduce come on top)
            proxy = {"dtype": bp}
            for n in (2, 4, 8):
                cls = args.classes // n
                log(f"batch1 class-shard proxy n{n} {bp}")
                trp, dmp = build_trainer(argparse.Namespace(**{**vars(args), "classes": cls}), bp, 1, dev, rank)
                # two timed rounds, the faster reported
                rounds = [time_train(trp, dmp, B1_STEPS, 5)[0] for _ in range(2)]
                proxy[f"n{n}"] = {"classes": cls, "ms_per_step": round(1000 * min(rounds) / B1_STEPS, 3),
                                  "rounds_ms": [round(1000 * t / B1_STEPS, 3) for t in rounds]}
                del trp, dmp
                torch.cuda.empty_cache()
            out["batch1_class_shard_proxy" + sfx] = proxy
        # BASELINE config 2: CoOp n_ctx 16, ViT-B/16 fp16, 1000 classes, batch 32 (the config names fp16)
        log("coop config 2")
        trc, dmc = build_coop_trainer(args, "fp16", 32, dev, rank, n_test_device=args.eval_images)
        tc, _ = time_train(trc, dmc, 10, 3)
        ec, nc = time_eval(trc, dmc, args.eval_images)
        out["coop"] = {"workload": f"CoOp {args.arch} n_ctx=16 end, {args.classes} classes, 32 images/GPU/step, "
                                   "fp16 (BASELINE config 2)", "images_per_sec": round(world * 32 * 10 / tc, 3),
                       "ms_per_step": round(100 * tc, 3), "eval_images_per_sec": round(ec, 3),
                       "eval_images": int(dist.sum_over_ranks(nc)),
                       "text_layout": ("shared-prefix packed" if trc.model.prompt_learner.layout.pack is not None
                                       else "plain")}
        del trc, dmc
        torch.cuda.empty_cache()
        # the other precisions at the headline workload: fp16 (the fastest mode, outside the 1e-3
        # bar; full eval set) and PREC fp32 (f32-input MFMA), or fp32s when it is not the headline
        for p in ("fp16", "fp32s", "fp32"):
            if p == args.prec:
                continue
            log(p)
            out[p] = precision_line(args, p, dev, rank, world, n_eval=args.eval_images if p != "fp32" else 5000)
        if args.weights == "fp16":
            # PREC fp32s on weights with fp32 mantissas (not a CLIP checkpoint: every GEMM keeps
            # the weight-lo product, split mode 1)
            log("fp32s, fp32-valued weights")
            out["fp32s_fp32_weights"] = precision_line(argparse.Namespace(**{**vars(args), "weights": "fp32"}),
                                                       "fp32s", dev, rank, world, n_eval=2000, prof=False)
    # after the ViT-B/16 lines: run before them, the ViT-L trainers left the launch-bound
    # 125-class proxy at 2.31 instead of 1.66-1.68 ms/step (same kernel durations; profiles/r05n)
    if not args.no_extra and args.arch in ("ViT-L/14", "ViT-L/14@336px"):
        out["config4" if args.arch == "ViT-L/14" else "config5"] = baseline_config_line(args, dev, rank, world)
    elif not args.no_extra and not args.no_configs and world == 1:
        # BASELINE configs 4 and 5 per GPU beside the headline (their own archs, bf16)
        for key, arch in (("config4", "ViT-L/14"), ("config5", "ViT-L/14@336px")):
            log(key)
            out[key] = baseline_config_line(argparse.Namespace(**{**vars(args), "arch": arch}), dev, rank, world,
                                            n_eval=2000)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            # the whole workload unit (1 image x all classes, fwd + bwd), no extrapolation (a
            # 50-class sample scaled linearly overstated the rate ~3x: the text activations of
            # 1,000 x 77 tokens do not stay in cache). SURVEY §8(d): the full host (every CPU this
            # process may run on) and an 8-thread run (the build container's reference timing)
            # "full host" = the CPU share this process is given: OMP_NUM_THREADS where the
            # launcher sets it (the GPU box: 16 of its nproc), else every CPU of the affinity set
            # (threads beyond the share oversubscribe it: 256 threads on a 16-CPU share ran
            # for minutes)
            aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
            host = int(os.environ.get("OMP_NUM_THREADS") or 0) or aff
            log(f"cpu baseline, {host} threads")
            cb = cpu_baseline(args.arch, "a photo of a", args.classes, args.cpu_classes or args.classes, host)
            cb["affinity_cpus"] = aff
            cb["share_note"] = "cores = OMP_NUM_THREADS (the process's CPU share) or the affinity set"
            log("cpu baseline, 8 threads")
            c8 = cpu_baseline(args.arch, "a photo of a", args.classes, args.cpu_classes or args.classes, 8)
            cb["eight_threads"] = {"value": c8["value"], "cores": 8}
            cb["reference"] = reference_cpu(args.arch, args.classes)
            out["cpu_baseline"] = cb
        except Exception as e:  # report, never fake
            out["cpu_baseline"] = {"value": None, "error": repr(e)}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist.is_dist():
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
