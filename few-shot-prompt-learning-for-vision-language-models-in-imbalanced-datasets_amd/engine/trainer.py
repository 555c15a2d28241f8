"""Trainer contract of Dassl's TrainerX (Dassl.pytorch/dassl/engine/trainer.py:77-303,
306-503, 596-650) for the CoOp/CoCoOp path: register_model / get_model_names /
update_lr / set_model_mode / save_model / resume / train / run_epoch / test /
model_inference, with the same checkpoint layout
(OUTPUT_DIR/<name>/model.pth.tar-<epoch> + ``checkpoint`` pointer, dict keys
state_dict/epoch/optimizer/scheduler/val_result; torchtools.py:27-157).

Multi-GPU: one process per GPU (torchrun); the learnable prompt gradients are
all-reduced over RCCL in ``allreduce_grads`` (fsp_amd.dist), replacing the reference's
nn.DataParallel wrap (coop.py:435-436, cocoop.py:308-311).
"""
from __future__ import annotations

import datetime
import os
import os.path as osp
import time
from collections import OrderedDict

import numpy as np
import torch

from .. import dist
from ..clip import synth
from ..clip.model import build_model
from .metrics import Classification


def load_clip(cfg, prec, device, text_grad=True):
    """Replacement for load_clip_to_cpu (coop.py:165-184): a local state dict from
    MODEL.WEIGHTS_PATH (torch.load weights_only=True / .npz / safetensors), otherwise
    the seeded synthetic CLIP of MODEL.BACKBONE.NAME (no network on this path).
    text_grad=False packs no backward weights (forward-only text encoder, e.g. zero-shot)."""
    path = cfg.MODEL.get("WEIGHTS_PATH", "")
    if path:
        if path.endswith(".npz"):
            with np.load(path, allow_pickle=False) as z:
                sd = {k: z[k] for k in z.files}
        elif path.endswith(".safetensors"):
            from safetensors.torch import load_file
            sd = load_file(path)
        else:
            sd = torch.load(path, map_location="cpu", weights_only=True)
            if "state_dict" in sd:
                sd = sd["state_dict"]
        sd = {k: v for k, v in sd.items() if k not in ("input_resolution", "context_length", "vocab_size")}
    else:
        sd = synth.make_state_dict(cfg.MODEL.BACKBONE.NAME, seed=0)
    return build_model(sd, prec=prec, device=device, text_grad=text_grad)


class TrainerX:
    def __init__(self, cfg, dm=None):
        self._models = OrderedDict()
        self._optims = OrderedDict()
        self._scheds = OrderedDict()
        self.cfg = cfg
        self.dm = dm
        self.device = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() \
            else torch.device("cpu")
        self.output_dir = cfg.OUTPUT_DIR
        self.start_epoch = self.epoch = 0
        self.max_epoch = cfg.OPTIM.MAX_EPOCH
        self.batch_idx = 0
        self.num_batches = 1
        self.check_cfg(cfg)
        self.build_model()
        self.evaluator = Classification(cfg, getattr(getattr(dm, "dataset", None), "lab2cname", None))
        self.best_result = -np.inf

    # ---- Dassl contract -------------------------------------------------------------
    def check_cfg(self, cfg):
        pass

    def build_model(self):
        raise NotImplementedError

    def forward_backward(self, batch):
        raise NotImplementedError

    def register_model(self, name="model", model=None, optim=None, sched=None):
        if name in self._models:
            raise KeyError("Cannot assign model with the same name")
        self._models[name] = model
        self._optims[name] = optim
        self._scheds[name] = sched

    def get_model_names(self, names=None):
        names_real = list(self._models.keys())
        if names is not None:
            names = [names] if isinstance(names, str) else names
            for n in names:
                assert n in names_real
            return names
        return names_real

    def update_lr(self, names=None):
        for n in self.get_model_names(names):
            if self._scheds[n] is not None:
                self._scheds[n].step()

    def get_current_lr(self, names=None):
        return self._optims[self.get_model_names(names)[0]].param_groups[0]["lr"]

    def set_model_mode(self, mode="train", names=None):
        for n in self.get_model_names(names):
            self._models[n].train() if mode == "train" else self._models[n].eval()
        self.model.train() if mode == "train" else self.model.eval()

    def allreduce_grads(self, module):
        dist.allreduce_grads([p for p in module.parameters() if p.requires_grad])

    def model_inference(self, x):
        return self.model(x)

    def parse_batch_test(self, batch):
        return batch["img"].to(self.device), batch["label"].to(self.device)

    # ---- checkpoints ----------------------------------------------------------------
    @staticmethod
    def load_checkpoint(path):
        return torch.load(path, map_location="cpu", weights_only=True)

    @staticmethod
    def load_pretrained_weights(module, path):
        ckpt = torch.load(path, map_location="cpu", weights_only=True)
        sd = ckpt.get("state_dict", ckpt)
        module.load_state_dict(sd, strict=False)

    def save_model(self, epoch, directory, is_best=False, val_result=None, model_name=""):
        if dist.rank() != 0:
            return
        for name in self.get_model_names():
            sd = {k: v.detach().cpu() for k, v in self._models[name].state_dict().items()}
            optim = self._optims[name].state_dict() if self._optims[name] is not None else None
            sched = self._scheds[name].state_dict() if self._scheds[name] is not None else None
            d = osp.join(directory, name)
            os.makedirs(d, exist_ok=True)
            fname = model_name or f"model.pth.tar-{epoch + 1}"
            torch.save({"state_dict": sd, "epoch": epoch + 1, "optimizer": optim, "scheduler": sched,
                        "val_result": val_result}, osp.join(d, fname))
            with open(osp.join(d, "checkpoint"), "w") as f:
                f.write(f"{fname}\n")
            if is_best:
                torch.save({"state_dict": sd, "epoch": epoch + 1, "optimizer": optim, "scheduler": sched,
                            "val_result": val_result}, osp.join(d, "model-best.pth.tar"))

    def resume_model_if_exist(self, directory):
        start = 0
        for name in self.get_model_names():
            d = osp.join(directory, name)
            ptr = osp.join(d, "checkpoint")
            if not osp.exists(ptr):
                return 0
            with open(ptr) as f:
                fname = f.readline().strip()
            ckpt = self.load_checkpoint(osp.join(d, fname))
            self._models[name].load_state_dict(ckpt["state_dict"])
            if ckpt.get("optimizer") and self._optims[name] is not None:
                self._optims[name].load_state_dict(ckpt["optimizer"])
            if ckpt.get("scheduler") and self._scheds[name] is not None:
                self._scheds[name].load_state_dict(ckpt["scheduler"])
            start = ckpt["epoch"]
        return start

    # ---- loops ----------------------------------------------------------------------
    def train(self, start_epoch=None, max_epoch=None):
        self.start_epoch = self.resume_model_if_exist(self.output_dir) if start_epoch is None else start_epoch
        self.max_epoch = self.max_epoch if max_epoch is None else max_epoch
        t0 = time.time()
        for self.epoch in range(self.start_epoch, self.max_epoch):
            self.run_epoch()
            self.save_model(self.epoch, self.output_dir)
        if not self.cfg.TEST.NO_TEST:
            self.test()
        print(f"Elapsed: {datetime.timedelta(seconds=round(time.time() - t0))}")

    def run_epoch(self):
        self.set_model_mode("train")
        loader = self.dm.train_loader_x
        self.num_batches = len(loader)
        for self.batch_idx, batch in enumerate(loader):
            summary = self.forward_backward(batch)
            if (self.batch_idx + 1) % self.cfg.TRAIN.PRINT_FREQ == 0 and dist.rank() == 0:
                print(f"epoch [{self.epoch + 1}/{self.max_epoch}] batch [{self.batch_idx + 1}/"
                      f"{self.num_batches}] {summary} lr {self.get_current_lr():.4e}")

    @torch.no_grad()
    def test(self, split="test", return_pred=False):
        self.set_model_mode("eval")
        self.evaluator.reset()
        loader = self.dm.test_loader if split == "test" else self.dm.val_loader
        for batch in loader:
            x, y = self.parse_batch_test(batch)
            out = self.model_inference(x)
            self.evaluator.process(out, y)
        results = self.evaluator.evaluate()
        return (results, self.evaluator.preds()) if return_pred else results
