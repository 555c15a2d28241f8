"""Trainer contract of Dassl's TrainerX (Dassl.pytorch/dassl/engine/trainer.py:77-303,
306-503, 596-650) for the CoOp/CoCoOp path: register_model / get_model_names /
update_lr / set_model_mode / save_model / resume_model_if_exist / load_model / train /
run_epoch / test / model_inference / parse_batch_test / get_current_lr, with the same
checkpoint layout (engine/checkpoint.py; torchtools.py:27-157) and the same ``test``
return contract (trainer.py:446-486: ``(y_true, y_pred)`` with ``return_pred``, else the
first metric).

Multi-GPU: one process per GPU (torchrun) instead of the reference's nn.DataParallel wrap
(coop.py:435-436, cocoop.py:308-311):
* the trainable prompt parameters are broadcast from rank 0 after ``build_model``, so
  every rank starts from the same ctx / Meta-Net whatever its seed;
* training batches come from a rank-aware loader (data/manager.py: every rank walks the
  same global sampler stream and takes its slice of each global batch), and the prompt
  gradients are all-reduced in ``allreduce_grads`` -- weighted by each rank's share of the
  global batch, so the update equals the single-process one on the union batch;
* ``test`` runs each rank on its shard of the test set and gathers (label, prediction)
  pairs, so every rank reports the metrics of the whole set.
"""
from __future__ import annotations

import datetime
import os.path as osp
import time
from collections import OrderedDict

import numpy as np
import torch

from .. import dist
from ..clip import synth
from ..clip.model import build_model
from ..clip.weights import load_state_dict
from . import checkpoint as ckpt
from .metrics import Classification


def load_clip(cfg, prec, device, text_grad=True, vision_grad=False):
    """Replacement for load_clip_to_cpu (coop.py:165-184): the CLIP weights file at
    MODEL.WEIGHTS_PATH (OpenAI TorchScript archive, torch.save state dict, .npz or
    .safetensors; clip/weights.py), otherwise the seeded synthetic CLIP of
    MODEL.BACKBONE.NAME (no network on this path). text_grad=False packs no backward
    weights (forward-only text encoder, e.g. zero-shot)."""
    path = cfg.MODEL.get("WEIGHTS_PATH", "")
    sd = load_state_dict(path) if path else synth.make_state_dict(
        cfg.MODEL.BACKBONE.NAME, seed=0, fp16_values=bool(cfg.MODEL.get("SYNTH_FP16", False)))
    return build_model(sd, prec=prec, device=device, text_grad=text_grad, vision_grad=vision_grad)


class TrainerX:
    def __init__(self, cfg, dm=None):
        self._models = OrderedDict()
        self._optims = OrderedDict()
        self._scheds = OrderedDict()
        self._writer = None
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
        self.sync_trainable()
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
            raise KeyError("Found duplicate model names")
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
            if mode == "train":
                self._models[n].train()
            elif mode in ("test", "eval"):
                self._models[n].eval()
            else:
                raise KeyError(mode)
        model = getattr(self, "model", None)
        if model is not None:
            model.train() if mode == "train" else model.eval()

    # ---- multi-GPU --------------------------------------------------------------------
    def trainable_params(self):
        return [p for n in self.get_model_names() for p in self._models[n].parameters() if p.requires_grad]

    def sync_trainable(self):
        """Broadcast the trainable parameters from rank 0 (no-op single-process)."""
        if dist.is_dist() and dist.world_size() > 1:
            dist.broadcast_params(self.trainable_params(), src=0)

    def allreduce_grads(self, module):
        # the average's 1 / world folded into the fused SGD step (FusedSGD.defer_grad_scale)
        dist.allreduce_grads([p for p in module.parameters() if p.requires_grad],
                             optimizer=getattr(self, "optim", None))

    @staticmethod
    def batch_weight(batch, n_local):
        """Scale for this rank's loss before backward, so that the averaged all-reduce
        gives the gradient of the mean loss over the global batch: n_local * world /
        n_global (1 when every rank holds an equal share). A batch marked ``n_local`` 0 is a
        pad (its rank's slice of a short last batch was empty, data/manager.py): weight 0,
        so it joins the all-reduce with a zero gradient."""
        if not isinstance(batch, dict):
            return 1.0
        n_global = batch.get("n_global")
        w = dist.world_size()
        if not n_global or w == 1:
            return 1.0
        n_local = batch.get("n_local", n_local)
        return float(n_local) * w / float(n_global)

    def model_inference(self, x):
        return self.model(x)

    def parse_batch_test(self, batch):
        return batch["img"].to(self.device), batch["label"].to(self.device)

    # ---- checkpoints ----------------------------------------------------------------
    @staticmethod
    def load_checkpoint(path):
        return ckpt.load_checkpoint(path)

    @staticmethod
    def load_pretrained_weights(module, path):
        """Dassl load_pretrained_weights (torchtools.py:267-314): matching keys and shapes."""
        ck = ckpt.load_checkpoint(path)
        sd = ck.get("state_dict", ck)
        own = module.state_dict()
        keep = {k[7:] if k.startswith("module.") else k: v for k, v in sd.items()}
        keep = {k: v for k, v in keep.items() if k in own and own[k].shape == v.shape}
        module.load_state_dict(keep, strict=False)

    def save_model(self, epoch, directory, is_best=False, val_result=None, model_name=""):
        self.flush_deferred()
        if dist.rank() != 0:
            return
        for name in self.get_model_names():
            sd = OrderedDict((k, v.detach().cpu()) for k, v in self._models[name].state_dict().items())
            optim = self._optims[name].state_dict() if self._optims[name] is not None else None
            sched = self._scheds[name].state_dict() if self._scheds[name] is not None else None
            ckpt.save_checkpoint({"state_dict": sd, "epoch": epoch + 1, "optimizer": optim, "scheduler": sched,
                                  "val_result": val_result}, osp.join(directory, name), is_best=is_best,
                                 model_name=model_name)

    def load_model(self, directory, epoch=None):
        """trainer.py:172-201 (the base form; CoOp / CoCoOp override it, dropping the token
        buffers): ``model-best.pth.tar`` by default, ``model.pth.tar-<epoch>`` when given."""
        if not directory:
            print("Note that load_model() is skipped as no pretrained model is given")
            return
        model_file = "model-best.pth.tar" if epoch is None else f"model.pth.tar-{epoch}"
        for name in self.get_model_names():
            model_path = osp.join(directory, name, model_file)
            if not osp.exists(model_path):
                raise FileNotFoundError(f"No model at {model_path}")
            ck = self.load_checkpoint(model_path)
            vr = ck.get("val_result")
            print(f"Load {model_path} to {name} (epoch={ck['epoch']}, val_result="
                  f"{vr if vr is None else format(vr, '.1f')})")
            self._models[name].load_state_dict(ck["state_dict"])

    def resume_model_if_exist(self, directory):
        names = self.get_model_names()
        if any(not osp.exists(osp.join(directory, n)) for n in names):
            print("No checkpoint found, train from scratch")
            return 0
        print(f"Found checkpoint at {directory} (will resume training)")
        start = 0
        for name in names:
            start = ckpt.resume_from_checkpoint(osp.join(directory, name), self._models[name],
                                                self._optims[name], self._scheds[name])
        return start

    # ---- loops ----------------------------------------------------------------------
    def train(self, start_epoch=None, max_epoch=None):
        """trainer.py:242-252 + before_train / after_train (388-420): resume from cfg.RESUME
        (else OUTPUT_DIR), the epoch loop, then the final test -- of the best-val model
        when TEST.FINAL_MODEL is "best_val"."""
        directory = self.cfg.get("RESUME", "") or self.output_dir
        self.start_epoch = self.resume_model_if_exist(directory) if start_epoch is None else start_epoch
        self.max_epoch = self.max_epoch if max_epoch is None else max_epoch
        t0 = time.time()
        for self.epoch in range(self.start_epoch, self.max_epoch):
            self.run_epoch()
            self.after_epoch()
        print("Finish training")
        if not self.cfg.TEST.NO_TEST:
            if self.cfg.TEST.get("FINAL_MODEL", "last_step") == "best_val":
                print("Deploy the model with the best val performance")
                # rank 0 alone writes model-best.pth.tar (save_model): every rank waits for it
                # before reading it back, so no rank loads a missing, partial or older file
                dist.barrier()
                self.load_model(self.output_dir)
            else:
                print("Deploy the last-epoch model")
            self.test()
        print(f"Elapsed: {datetime.timedelta(seconds=round(time.time() - t0))}")

    def after_epoch(self):
        """trainer.py:422-443: with TEST.FINAL_MODEL "best_val" a val test every epoch and
        ``model-best.pth.tar`` whenever it improves; a checkpoint at CHECKPOINT_FREQ and at
        the last epoch."""
        last = (self.epoch + 1) == self.max_epoch
        freq = self.cfg.TRAIN.get("CHECKPOINT_FREQ", 0)
        if not self.cfg.TEST.NO_TEST and self.cfg.TEST.get("FINAL_MODEL", "last_step") == "best_val":
            curr = self.test(split="val")
            if curr > self.best_result:
                self.best_result = curr
                self.save_model(self.epoch, self.output_dir, val_result=curr, model_name="model-best.pth.tar")
        if last or (freq > 0 and (self.epoch + 1) % freq == 0):
            self.save_model(self.epoch, self.output_dir)

    def run_epoch(self):
        self.set_model_mode("train")
        dist.sync_rng_from(0)  # one global sampler stream on every rank (data/manager.py)
        loader = self.dm.train_loader_x
        self.num_batches = len(loader)
        # one batch of lookahead: forward_backward may start work on the next batch (CoCoOp's
        # frozen image encoder, NATIVE.PREFETCH_VISION); the batches and their order are unchanged
        it = iter(loader)
        batch = next(it, None)
        self.batch_idx = -1
        while batch is not None:
            nxt = next(it, None)
            self.batch_idx += 1
            self.next_batch = nxt
            summary = self.forward_backward(batch)
            batch = nxt
            if (self.batch_idx + 1) % self.cfg.TRAIN.PRINT_FREQ == 0 and dist.rank() == 0:
                print(f"epoch [{self.epoch + 1}/{self.max_epoch}] batch [{self.batch_idx + 1}/"
                      f"{self.num_batches}] {summary} lr {self.get_current_lr():.4e}")
        self.flush_deferred()

    def flush_deferred(self):
        """Settle a check the last step left pending (PREC fp32s, CoCoOp.forward_backward); a
        no-op for trainers that check in the step."""

    @torch.no_grad()
    def test(self, split=None, return_pred=False):
        """trainer.py:446-486. Each rank evaluates its shard of the split (the loader is
        rank-aware); labels and predictions are gathered so every rank evaluates the union.
        Returns (y_true, y_pred) numpy arrays with ``return_pred``, else the first metric."""
        self.flush_deferred()
        self.set_model_mode("eval")
        self.evaluator.reset()
        if split is None:
            split = self.cfg.TEST.get("SPLIT", "test")
        val = getattr(self.dm, "val_loader", None)
        if split == "val" and val is not None:
            loader = val
        else:
            split = "test"
            loader = self.dm.test_loader
        print(f"Evaluate on the *{split}* set")
        prepare = getattr(self.model, "prepare_eval", None)
        if prepare is not None:  # every rank joins its collectives, whatever its shard size
            prepare()
        preds, labels = [], []
        # one batch of lookahead: the model may start the next batch's image encoder meanwhile
        # (CoCoOp, NATIVE.PREFETCH_VISION); results do not depend on it
        hint = hasattr(self.model, "prefetch_image_features")
        it = iter(loader)
        batch = next(it, None)
        while batch is not None:
            nxt = next(it, None)
            x, y = self.parse_batch_test(batch)
            if hint:
                self.model.next_image = self.parse_batch_test(nxt)[0] if nxt is not None else None
            out = self.model_inference(x)
            batch = nxt
            preds.append(out.argmax(1).to(torch.int64))
            labels.append(y.to(torch.int64))
        # PREC fp32s: the inference forwards' overflow flags, read once here (clip.model.SplitStatus)
        from ..clip.model import check_split_status
        check_split_status(self.device)
        dev = self.device
        p = torch.cat(preds) if preds else torch.zeros(0, dtype=torch.int64, device=dev)
        y = torch.cat(labels) if labels else torch.zeros(0, dtype=torch.int64, device=dev)
        if not dist.batches_replicated(self.cfg):  # replicated: every rank saw the whole split
            p, y = dist.all_gather_varlen(p), dist.all_gather_varlen(y)
        y_true, y_pred = y.cpu().numpy(), p.cpu().numpy()
        results = self.evaluator.evaluate_arrays(y_true, y_pred)
        if return_pred:
            return y_true, y_pred
        return list(results.values())[0]
