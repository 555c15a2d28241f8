"""Shared prompt-learner machinery for CoOp and CoCoOp.

Both reference learners build ``token_prefix`` = emb[:, :1] and ``token_suffix`` =
emb[:, 1+n_ctx:] from ``token_embedding(tokenize(prompts))`` (coop.py:236-257,
cocoop.py:149-162) and splice context vectors in between. Here the same buffers are
kept (checkpoint compatibility) and, for the native path, a [C,77,W] embedding table
with the context slots zeroed plus the int32 slot tables consumed by
``clipk_prompt_assemble`` / ``clipk_ctx_grad``.
"""
from __future__ import annotations

import os

import numpy as np
import torch
import torch.nn as nn

from ..clip.tokenizer import tokenize, default_tokenizer
from ._fns import prompt_layout


def grads_finite(module) -> bool:
    """GradScaler.step's skip test (inf / nan in any gradient); one host sync."""
    gs = [p.grad for p in module.parameters() if p.grad is not None]
    if not gs:
        return True
    return bool(torch.stack([torch.isfinite(g).all() for g in gs]).all().item())


# prefix-input mode on packed layouts whose trainable slots all sit in the shared prefix
# (knob CLIPK_TEXT_PREFIX_INPUT=0 turns it off; A/B and parity on both)
PREFIX_INPUT = os.environ.get("CLIPK_TEXT_PREFIX_INPUT", "1") != "0"


class TextShape:
    """Row structure of one text-encoder call, as the native encoder takes it.

    plain : nseq sequences of L rows (row s*L + t), eot_rows[s] = s*L + EOT_s.
    packed: G groups of R rows sharing a P-row causal prefix (see shared_prefix_tables);
            tiles [ntiles,2] int32 (first row, rows) of the <=16-row attention tiles,
            row_first [R] int32, eot_rows[g*C + c] absolute."""

    def __init__(self, eot_rows, nseq=0, L=0, G=0, C=0, P=0, R=0, tiles=None, row_first=None,
                 prefix_input=False):
        self.eot_rows = eot_rows
        # packed only: every trainable slot is a prefix row, so the class rows of x0 are the
        # same in every group and the input gradient is wanted on the prefix rows alone
        # (clipk_encoder_set_input_rows; dx0's class rows are then unspecified)
        self.prefix_input = bool(prefix_input) and tiles is not None
        self.packed = tiles is not None
        self.nseq, self.L = nseq, L
        self.G, self.C, self.P, self.R = G, C, P, R
        self.tiles, self.row_first = tiles, row_first
        self.ntiles = 0 if tiles is None else tiles.numel() // 2
        self.rows = G * R if self.packed else nseq * L
        self.nout = G * C if self.packed else nseq


def attention_tiles(off, qlen, R, max_rows=16):
    """Attention work tiles of the packed layout: consecutive whole classes packed greedily
    into windows of <= max_rows rows (so one 16-row MFMA tile carries ~16/q_len classes).
    Returns (tiles [ntiles, 2] int32 = (first row, rows), row_first [R] int32 = first row of
    each row's class; 0 for the prefix rows)."""
    tiles, t0, rows = [], int(off[0]), 0
    for c in range(len(qlen)):
        if rows + int(qlen[c]) > max_rows:
            tiles.append((t0, rows))
            t0, rows = int(off[c]), 0
        rows += int(qlen[c])
    tiles.append((t0, rows))
    row_first = np.zeros(R, np.int32)
    for c in range(len(qlen)):
        row_first[off[c]:off[c] + qlen[c]] = off[c]
    return np.asarray(tiles, np.int32), row_first


def shared_prefix_tables(src_map, ctx_pos, eot, n_ctx, csc, max_prefix=16, max_q=16):
    """Packing tables for the shared causal prefix (attention_prefix.hip), or None.

    The structural prefix = SOT + the context slots before the first class-name token
    (position "end": 1 + n_ctx, "middle": 1 + n_ctx/2, "front": 1), identical for every
    class when the context is shared (not CSC). Coincidentally equal class-name tokens are
    NOT folded in, so the row count does not depend on the class-name vocabulary.
    Under the causal mask those rows' states are the same for every class, and rows past a
    class's EOT never reach its EOT row: packing [prefix][class rows P..EOT_c]... is exact."""
    C, L = src_map.shape
    if csc or n_ctx <= 0:
        return None
    P = 1
    while P < L and src_map[0, P] < 0 and (src_map[:, P] == src_map[0, P]).all():
        P += 1
    P = min(P, max_prefix)
    qlen = np.asarray(eot, np.int64) + 1 - P
    if P < 2 or qlen.min() < 1 or qlen.max() > max_q:
        return None
    off = P + np.concatenate([[0], np.cumsum(qlen)[:-1]])
    R = int(P + qlen.sum())
    row_tab = np.empty(R, np.int32)
    row_tab[:P] = np.arange(P)
    for c in range(C):
        row_tab[off[c]:off[c] + qlen[c]] = c * L + np.arange(P, P + qlen[c])
    slot_ptr = [0]
    slot_rows = []
    for k in range(n_ctx):
        t0 = int(ctx_pos[0, k])
        if t0 < P and (ctx_pos[:, k] == t0).all():
            slot_rows.append(t0)
        else:
            slot_rows.extend(int(off[c] + ctx_pos[c, k] - P) for c in range(C))
        slot_ptr.append(len(slot_rows))
    seg = np.stack([off, qlen], 1).astype(np.int32)
    tiles, row_first = attention_tiles(off, qlen, R, max_q)
    return {"P": P, "R": R, "seg": seg, "row_tab": row_tab, "max_q": int(qlen.max()),
            "tiles": np.asarray(tiles, np.int32), "row_first": row_first,
            "slot_ptr": np.asarray(slot_ptr, np.int32), "slot_rows": np.asarray(slot_rows, np.int32),
            "eot_in_group": (off + qlen - 1).astype(np.int64)}


class PromptLayout:
    """Device-resident slot tables for one (class set, n_ctx, position)."""

    def __init__(self, n_cls, n_ctx, src_map, ctx_pos, L, eot, emb, pos, csc=False, shared_prefix=True):
        self.n_cls, self.n_ctx, self.L = n_cls, n_ctx, L
        dev = emb.device
        self.src_map = torch.from_numpy(src_map).to(dev)
        self.ctx_pos = torch.from_numpy(ctx_pos).to(dev)
        self.eot = np.asarray(eot, np.int64)
        self.emb = emb
        self.pos = pos.contiguous()
        self._eot_rows = {}
        self._shapes = {}
        pk = shared_prefix_tables(src_map, ctx_pos, eot, n_ctx, csc) if shared_prefix else None
        self.pack = None
        self.prefix_input = False
        if pk is not None:
            self.pack = pk
            self.P, self.R = pk["P"], pk["R"]
            self.tiles = torch.from_numpy(pk["tiles"].reshape(-1).copy()).to(dev)
            self.row_first = torch.from_numpy(pk["row_first"]).to(dev)
            self.row_tab = torch.from_numpy(pk["row_tab"]).to(dev)
            self.slot_ptr = torch.from_numpy(pk["slot_ptr"]).to(dev)
            self.slot_rows = torch.from_numpy(pk["slot_rows"]).to(dev)
            self.prefix_input = len(pk["slot_rows"]) == n_ctx and bool((pk["slot_rows"] < self.P).all())

    @property
    def rows_per_group(self) -> int:
        """Text rows one image (CoCoOp) / the class set (CoOp) costs."""
        return self.R if self.pack is not None else self.n_cls * self.L

    def eot_rows(self, B: int) -> torch.Tensor:
        """Global row index of each sequence's EOT token, ordered (b, c)."""
        if B not in self._eot_rows:
            b = np.arange(B)[:, None]
            if self.pack is not None:
                rows = b * self.R + self.pack["eot_in_group"][None, :]
            else:
                rows = (b * self.n_cls + np.arange(self.n_cls)[None, :]) * self.L + self.eot[None, :]
            self._eot_rows[B] = torch.from_numpy(rows.reshape(-1).astype(np.int32)).to(self.emb.device)
        return self._eot_rows[B]

    def shape(self, B: int) -> TextShape:
        """TextShape for B groups (images for CoCoOp; 1 for CoOp)."""
        if B not in self._shapes:
            if self.pack is not None:
                self._shapes[B] = TextShape(self.eot_rows(B), G=B, C=self.n_cls, P=self.P, R=self.R,
                                            tiles=self.tiles, row_first=self.row_first,
                                            prefix_input=self.prefix_input and PREFIX_INPUT)
            else:
                self._shapes[B] = TextShape(self.eot_rows(B), nseq=B * self.n_cls, L=self.L)
        return self._shapes[B]


def init_prompts(module: nn.Module, classnames, clip_model, n_ctx, ctx_init, position, csc,
                 truncate: bool, shared_prefix: bool = True, class_range=None, vl_init: bool = False):
    """Common __init__ body; returns (ctx_vectors, prompt_prefix).

    class_range (lo, hi): the native layout covers only classes [lo, hi) -- this rank's
    shard under class-sharded text encoding (CoOp); the checkpointed buffers
    (token_prefix / token_suffix) and ``n_cls`` still cover every class.
    vl_init: the IVLP / MaPLe / PromptSRC rule (independentVL.py:205-215, maple.py:128-137):
    CTX_INIT is used only when N_CTX <= 4, and then N_CTX (not the word count) context
    vectors come from its first tokens while the prompt text keeps all its words."""
    n_cls = len(classnames)
    W = clip_model.arch.transformer_width
    dev = clip_model.positional_embedding.device
    emb_layer = clip_model.token_embedding
    if ctx_init and (not vl_init or n_ctx <= 4):
        ctx_init = ctx_init.replace("_", " ")
        if not vl_init:
            n_ctx = len(ctx_init.split(" "))
        prompt = torch.from_numpy(tokenize(ctx_init))
        with torch.no_grad():
            embedding = emb_layer(prompt)
        ctx_vectors = embedding[0, 1:1 + n_ctx, :].clone()
        prompt_prefix = ctx_init
    else:
        shape = (n_cls, n_ctx, W) if csc else (n_ctx, W)
        ctx_vectors = torch.empty(*shape)
        nn.init.normal_(ctx_vectors, std=0.02)
        prompt_prefix = " ".join(["X"] * n_ctx)
    print(f'Initial context: "{prompt_prefix}"')
    print(f"Number of context words (tokens): {n_ctx}")
    names = [name.replace("_", " ") for name in classnames]
    tok = default_tokenizer()
    name_lens = [len(tok.encode(name)) for name in names]
    prompts = [prompt_prefix + " " + name + "." for name in names]
    tokenized = torch.from_numpy(tokenize(prompts))
    with torch.no_grad():
        embedding = emb_layer(tokenized).float()
    module.register_buffer("token_prefix", embedding[:, :1, :].to(dev))
    module.register_buffer("token_suffix", embedding[:, 1 + n_ctx:, :].to(dev))
    emb = embedding.clone()
    emb[:, 1:1 + n_ctx] = 0.0
    eot = tokenized.argmax(dim=-1).numpy()
    src, cpos, L = prompt_layout(n_cls, n_ctx, name_lens, position, eot, truncate)
    lo, hi = (0, n_cls) if class_range is None else class_range
    module.class_range = (lo, hi)
    module.layout = PromptLayout(hi - lo, n_ctx, src[lo:hi], cpos[lo:hi], L, eot[lo:hi],
                                 emb[lo:hi].to(dev).contiguous(), clip_model.positional_embedding.detach(),
                                 csc=csc, shared_prefix=shared_prefix and truncate)
    module.n_cls, module.n_ctx = n_cls, n_ctx
    module.tokenized_prompts = tokenized
    module.name_lens = name_lens
    return ctx_vectors.to(dev), prompt_prefix
