"""Config surface for the CoOp/CoCoOp path (yacs is not in the image).

``CfgNode`` keeps the yacs behaviours the reference relies on: attribute access, ``get``,
``merge_from_file`` (YAML), ``merge_from_list`` (CLI ``KEY VAL`` pairs), ``freeze``.
Defaults cover the keys the CoOp/CoCoOp hot path reads: Dassl defaults
(Dassl.pytorch/dassl/config/defaults.py) for INPUT/DATASET/DATALOADER/OPTIM/MODEL and
``extend_cfg`` (PromptSRC/train.py:88-114,195) for TRAINER.COOP / TRAINER.COCOOP.
"""
from __future__ import annotations

import ast
import copy

import yaml


class CfgNode(dict):
    def __init__(self, init=None):
        super().__init__()
        object.__setattr__(self, "_frozen", False)
        for k, v in (init or {}).items():
            self[k] = CfgNode(v) if isinstance(v, dict) and not isinstance(v, CfgNode) else v

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e

    def __setattr__(self, k, v):
        if self._frozen:
            raise AttributeError(f"Attempted to set {k} on a frozen CfgNode")
        self[k] = v

    def freeze(self):
        object.__setattr__(self, "_frozen", True)
        for v in self.values():
            if isinstance(v, CfgNode):
                v.freeze()

    def defrost(self):
        object.__setattr__(self, "_frozen", False)
        for v in self.values():
            if isinstance(v, CfgNode):
                v.defrost()

    def clone(self):
        c = CfgNode(copy.deepcopy(dict(self)))
        return c

    def _merge(self, other, path=""):
        for k, v in other.items():
            if k not in self:
                self[k] = CfgNode(v) if isinstance(v, dict) else v  # new keys allowed (extend_cfg style)
                continue
            if isinstance(self[k], CfgNode) and isinstance(v, dict):
                self[k]._merge(v, path + k + ".")
            else:
                self[k] = _coerce(self[k], v, path + k)

    def merge_from_file(self, path):
        with open(path) as f:
            self._merge(yaml.safe_load(f) or {})

    def merge_from_list(self, opts):
        if len(opts) % 2:
            raise ValueError("opts must be KEY VALUE pairs")
        for key, val in zip(opts[0::2], opts[1::2]):
            node = self
            parts = key.split(".")
            for p in parts[:-1]:
                node = node[p]
            try:
                v = ast.literal_eval(val) if isinstance(val, str) else val
            except (ValueError, SyntaxError):
                v = val
            node[parts[-1]] = _coerce(node.get(parts[-1]), v, key)


def _coerce(old, new, key):
    if old is None or new is None:
        return new
    if isinstance(old, tuple) and isinstance(new, list):
        return tuple(new)
    if isinstance(old, bool) and isinstance(new, str):
        return new.lower() in ("1", "true", "yes")
    if isinstance(old, float) and isinstance(new, int) and not isinstance(new, bool):
        return float(new)
    if isinstance(old, str) and not isinstance(new, str):
        return str(new)
    return new


def get_cfg_default() -> CfgNode:
    return CfgNode({
        "OUTPUT_DIR": "./output",
        "RESUME": "",
        "SEED": -1,
        "USE_CUDA": True,
        "INPUT": {"SIZE": (224, 224), "INTERPOLATION": "bicubic",
                  "PIXEL_MEAN": [0.48145466, 0.4578275, 0.40821073],
                  "PIXEL_STD": [0.26862954, 0.26130258, 0.27577711],
                  "TRANSFORMS": ["random_resized_crop", "random_flip", "normalize"]},
        "DATASET": {"ROOT": "", "NAME": "", "NUM_SHOTS": -1, "PER_CLASS_SHOTS": [],
                    "SUBSAMPLE_CLASSES": "all"},
        "DATALOADER": {"NUM_WORKERS": 8, "TRAIN_X": {"SAMPLER": "RandomSampler", "BATCH_SIZE": 32},
                       "TEST": {"SAMPLER": "SequentialSampler", "BATCH_SIZE": 100}},
        "MODEL": {"INIT_WEIGHTS": "", "BACKBONE": {"NAME": "ViT-B/16"}, "WEIGHTS_PATH": "",
                  "SYNTH_FP16": False},
        "OPTIM": {"NAME": "sgd", "LR": 0.002, "WEIGHT_DECAY": 5e-4, "MOMENTUM": 0.9,
                  "SGD_DAMPNING": 0, "SGD_NESTEROV": False, "LR_SCHEDULER": "cosine",
                  "MAX_EPOCH": 10, "WARMUP_EPOCH": -1, "WARMUP_TYPE": "linear",
                  "WARMUP_CONS_LR": 1e-5, "WARMUP_MIN_LR": 1e-5, "WARMUP_RECOUNT": True},
        "TRAIN": {"PRINT_FREQ": 10, "CHECKPOINT_FREQ": 0},
        "TEST": {"EVALUATOR": "Classification", "FINAL_MODEL": "last_step", "NO_TEST": False,
                 "SPLIT": "test"},
        "TRAINER": {
            "NAME": "",
            # PromptSRC/train.py:101-108
            "COOP": {"N_CTX": 16, "CSC": False, "CTX_INIT": "", "PREC": "fp16",
                     "CLASS_TOKEN_POSITION": "end", "USE_FOCAL_LOSS": False, "LOSS_TYPE": "ce"},
            # PromptSRC/train.py:110-114
            "COCOOP": {"N_CTX": 16, "CTX_INIT": "", "PREC": "fp16", "USE_FOCAL_LOSS": False},
            # PromptSRC/train.py:116-122
            "MAPLE": {"N_CTX": 2, "CTX_INIT": "a photo of a", "PREC": "fp16", "PROMPT_DEPTH": 9,
                      "USE_FOCAL_LOSS": False},
            # PromptSRC/train.py:125-141 (+ LOGITS_LOSS_WEIGHT and USE_GPA, which the trainer
            # reads, promptsrc.py:320, 330, but train.py never defines)
            "PROMPTSRC": {"N_CTX_VISION": 4, "N_CTX_TEXT": 4, "CTX_INIT": "a photo of a", "PREC": "fp16",
                          "PROMPT_DEPTH_VISION": 9, "PROMPT_DEPTH_TEXT": 9, "TEXT_LOSS_WEIGHT": 25,
                          "IMAGE_LOSS_WEIGHT": 10, "LOGITS_LOSS_WEIGHT": 1.0, "GPA_MEAN": 15, "GPA_STD": 1,
                          "USE_GPA": True, "LABEL_SCOPE": "default", "LOSS_TYPE": "ce", "SIMCLR_ALPHA": 0.0},
            # PromptSRC/train.py:144-159. USE_KD defaults off here: its teacher is a pretrained
            # timm download (independentVL.py:360-365), which this path cannot fetch.
            "IVLP": {"N_CTX_VISION": 2, "N_CTX_TEXT": 2, "CTX_INIT": "a photo of a", "PREC": "fp16",
                     "PROMPT_DEPTH_VISION": 9, "PROMPT_DEPTH_TEXT": 9, "USE_FOCAL_LOSS": False,
                     "SIMCLR_ALPHA": 0.0, "USE_MIXUP": True, "MIXUP_ALPHA": 1.0, "USE_KD": False,
                     "KD_TEACHER_MODEL": "resnet50", "KD_ALPHA": 1.0, "KD_T": 4.0},
        },
        # MI355X-native knobs (not in the reference): prompt truncation to the EOT and the
        # max rows per text-encoder launch chunk (memory bound for large B*C).
        # CLASS_SHARD: CoOp under torchrun encodes C / world classes per rank.
        # COCOOP_SHARD: CoCoOp under torchrun, "image" (data parallel) or "class" (every rank
        # scores the same batch against C / world classes; SURVEY §8(e) Option B).
        "NATIVE": {"TRUNCATE_PROMPTS": True, "SHARED_PREFIX": True, "MAX_TEXT_ROWS": 2_000_000,
                   "CLASS_SHARD": True, "COCOOP_SHARD": "image",
                   # OVERLAP_VISION: CoOp runs the frozen image encoder on a side stream while the
                   # text encoder (independent of the images) runs on the main one
                   "OVERLAP_VISION": True,
                   # PREFETCH_VISION: CoCoOp starts the next batch's image encoder (frozen) on a side
                   # stream between a step's forward and backward (the loop names the next batch)
                   "PREFETCH_VISION": True,
                   # DEFER_SPLIT_CHECK: PREC fp32s CoCoOp (one process) reads a step's overflow flag
                   # in the next step instead of waiting for it in the backward (same updates:
                   # CoCoOp.forward_backward)
                   "DEFER_SPLIT_CHECK": True},
    })
