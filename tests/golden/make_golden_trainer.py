"""Trainer-level golden vectors from the REFERENCE trainers (run in the build container only:
needs /root/reference).

    python tests/golden/make_golden_trainer.py

Runs the reference CoOp / CoCoOp TRAINERS (PromptSRC/trainers/{coop,cocoop}.py on top of the
real Dassl TrainerX / SimpleTrainer / TrainerBase, dassl/engine/trainer.py loaded by path)
on the tiny seeded CLIP (fsp_amd.clip.synth; fp32, CPU):
* ``run_epoch`` for MAX_EPOCH epochs of 2 batches -- forward_backward with CoOp's post-step
  acc re-forward (coop.py:464-469) and ``update_lr`` at the last batch of each epoch;
* ``save_model`` -> the reference's own ``save_checkpoint`` (torchtools.py:27-74), whose
  scheduler entry pickles Dassl's ConstantWarmupScheduler successor;
* ``test(return_pred=True)`` and ``test()`` (trainer.py:446-486).
Recorded: per-step loss (and acc), the LR after each epoch, ctx / Meta-Net after training, the
test logits, (y_true, y_pred), the returned accuracy, and the checkpoint directory itself
(tests/golden/ref_ckpt_<trainer>/prompt_learner/...).

Stand-ins (modules the image lacks; none is on the computed path): ``torch.utils.tensorboard``
(SummaryWriter never created: the writer stays None), ``dassl.data`` / ``dassl.modeling``
(DataManager / SimpleNet backbones, unused by CoOp/CoCoOp), plus make_golden.py's ftfy /
torchvision stand-ins; ``load_clip_to_cpu`` returns the reference ``build_model`` of the seeded
state dict (no download). Dassl's scheduler passes ``verbose`` positionally, which torch 2.10
rejects: the same one-line ``_LRScheduler.__init__`` shim as make_golden.py's LR fixture.
"""
from __future__ import annotations

import importlib.util
import json
import os
import shutil
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)

import make_golden as MG  # noqa: E402
from fsp_amd.clip import synth  # noqa: E402
from fsp_amd.engine.config import get_cfg_default  # noqa: E402

ARCH, N_CLS, BATCH, N_BATCHES, EPOCHS = "tiny", 5, 3, 2, 2


def install_real_trainer():
    MG._install_stubs()  # ftfy, torchvision, dassl.engine stand-in (replaced below)
    tb = types.ModuleType("torch.utils.tensorboard")

    class SummaryWriter:  # never constructed on this path
        def __init__(self, *a, **k):
            raise RuntimeError("tensorboard is not available")

    tb.SummaryWriter = SummaryWriter
    sys.modules["torch.utils.tensorboard"] = tb
    dd = types.ModuleType("dassl.data")
    dd.DataManager = object
    sys.modules["dassl.data"] = dd
    dm = types.ModuleType("dassl.modeling")
    dm.build_head = dm.build_backbone = None
    sys.modules["dassl.modeling"] = dm
    spec = importlib.util.spec_from_file_location("dassl.engine.trainer",
                                                  os.path.join(MG.DASSL, "dassl", "engine", "trainer.py"))
    mod = importlib.util.module_from_spec(spec)
    sys.modules["dassl.engine.trainer"] = mod
    spec.loader.exec_module(mod)
    eng = sys.modules["dassl.engine"]
    eng.TrainerX = mod.TrainerX
    from dassl.optim import lr_scheduler as ls
    base = torch.optim.lr_scheduler.LRScheduler.__init__

    def init(self, optimizer, last_epoch=-1, verbose=False):
        base(self, optimizer, last_epoch)

    ls._LRScheduler.__init__ = init
    return mod


def make_cfg(trainer, outdir):
    cfg = get_cfg_default()
    a = synth.ARCHS[ARCH]
    cfg.OUTPUT_DIR = outdir
    cfg.INPUT.SIZE = (a.image_resolution, a.image_resolution)
    cfg.MODEL.BACKBONE.NAME = ARCH
    cfg.OPTIM.MAX_EPOCH = EPOCHS
    cfg.OPTIM.WARMUP_EPOCH = 1
    cfg.OPTIM.WARMUP_TYPE = "constant"
    cfg.OPTIM.WARMUP_CONS_LR = 1e-5
    cfg.OPTIM.LR = 0.002
    # Dassl optimizer/evaluator keys the reference reads
    cfg.OPTIM.update({"RMSPROP_ALPHA": 0.99, "ADAM_BETA1": 0.9, "ADAM_BETA2": 0.999, "STAGED_LR": False,
                      "NEW_LAYERS": (), "BASE_LR_MULT": 0.1, "STEPSIZE": (-1,), "GAMMA": 0.1})
    cfg.TEST.update({"PER_CLASS_RESULT": False, "COMPUTE_CMAT": False})
    cfg.TRAIN.PRINT_FREQ = 1
    cfg.VERBOSE = False
    cfg.TRAINER.NAME = trainer
    if trainer == "CoOp":
        c = cfg.TRAINER.COOP
        c.N_CTX, c.CTX_INIT, c.CSC, c.CLASS_TOKEN_POSITION, c.PREC, c.LOSS_TYPE = 4, "", False, "end", "fp32", "ce"
    else:
        c = cfg.TRAINER.COCOOP
        c.N_CTX, c.CTX_INIT, c.PREC, c.USE_FOCAL_LOSS = 4, "a photo of a", "fp32", False
    return cfg


def batches():
    a = synth.ARCHS[ARCH]
    train = []
    for i in range(N_BATCHES):
        img = torch.from_numpy(synth.make_images(BATCH, a.image_resolution, seed=100 + i))
        lbl = torch.from_numpy(synth.make_labels(BATCH, N_CLS, seed=200 + i))
        train.append({"img": img, "label": lbl, "domain": torch.zeros(BATCH, dtype=torch.int64)})
    test = []
    for i in range(2):
        img = torch.from_numpy(synth.make_images(4, a.image_resolution, seed=300 + i))
        lbl = torch.from_numpy(synth.make_labels(4, N_CLS, seed=400 + i))
        test.append({"img": img, "label": lbl})
    return train, test


def run(trainer_name):
    tmod = install_real_trainer()
    from clip.model import build_model
    mod = __import__(f"trainers.{trainer_name.lower()}", fromlist=["x"])
    outdir = os.path.join(HERE, f"ref_ckpt_{trainer_name.lower()}")
    shutil.rmtree(outdir, ignore_errors=True)
    cfg = make_cfg(trainer_name, outdir)
    sd, digest = MG.build_clip(ARCH)
    mod.load_clip_to_cpu = lambda cfg_: build_model(dict(sd), dict(MG.DESIGN, trainer=trainer_name)).float()
    cls = getattr(mod, trainer_name)
    tr = cls.__new__(cls)
    tmod.TrainerBase.__init__(tr)
    tr.cfg = cfg
    tr.device = torch.device("cpu")
    names = synth.synthetic_classnames(N_CLS)
    tr.dm = types.SimpleNamespace(dataset=types.SimpleNamespace(classnames=names,
                                                                lab2cname={i: n for i, n in enumerate(names)}))
    tr.output_dir, tr.start_epoch, tr.epoch, tr.max_epoch = outdir, 0, 0, EPOCHS
    tr.build_model()
    from dassl.evaluation import build_evaluator
    tr.evaluator = build_evaluator(cfg, lab2cname=tr.dm.dataset.lab2cname)
    pl = tr.model.prompt_learner
    a = synth.ARCHS[ARCH]
    with torch.no_grad():
        if trainer_name == "CoOp":
            pl.ctx.copy_(torch.from_numpy(synth.make_ctx(4, a.transformer_width, seed=3)))
        else:
            mn = synth.make_meta_net(a.embed_dim, a.transformer_width, seed=4)
            for k, v in mn.items():
                dict(pl.named_parameters())[k].copy_(torch.from_numpy(v))
    ctx0 = pl.ctx.detach().clone().numpy()
    train, test = batches()
    tr.train_loader_x = train
    tr.test_loader = test
    tr.val_loader = None
    steps = []
    fb = tr.forward_backward

    def record(batch):
        out = fb(batch)
        steps.append(dict(out))
        return out

    tr.forward_backward = record
    lrs = []
    for tr.epoch in range(EPOCHS):
        tr.run_epoch()
        lrs.append(tr.get_current_lr())
    tr.save_model(tr.epoch, outdir)
    tr.set_model_mode("eval")
    with torch.no_grad():
        logits = torch.cat([tr.model_inference(b["img"]) for b in test]).numpy()
    y_true, y_pred = tr.test(return_pred=True)
    acc = tr.test()
    arrays = {"ctx0": ctx0, "ctx_final": pl.ctx.detach().numpy(),
              "loss": np.asarray([s["loss"] for s in steps], np.float64),
              "lr_after_epoch": np.asarray(lrs, np.float64), "test_logits": logits,
              "y_true": np.asarray(y_true), "y_pred": np.asarray(y_pred)}
    if "acc" in steps[0]:
        arrays["acc"] = np.asarray([s["acc"] for s in steps], np.float64)
    for k, p in pl.named_parameters():
        if k.startswith("meta_net"):
            arrays["final_" + k] = p.detach().numpy()
    meta = {"arch": ARCH, "digest": digest, "trainer": trainer_name, "n_cls": N_CLS, "batch": BATCH,
            "n_batches": N_BATCHES, "epochs": EPOCHS, "test_acc": float(acc),
            "ckpt": f"ref_ckpt_{trainer_name.lower()}/prompt_learner/model.pth.tar-{EPOCHS}"}
    np.savez_compressed(os.path.join(HERE, f"trainer_{trainer_name.lower()}.npz"), meta=json.dumps(meta), **arrays)
    print("wrote", trainer_name, meta, {k: v.shape for k, v in arrays.items()})


if __name__ == "__main__":
    torch.set_num_threads(8)
    which = sys.argv[1:] or ["CoOp", "CoCoOp"]
    for t in which:
        run(t)
