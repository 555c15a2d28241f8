"""Shared prompt-learner machinery for CoOp and CoCoOp.

Both reference learners build ``token_prefix`` = emb[:, :1] and ``token_suffix`` =
emb[:, 1+n_ctx:] from ``token_embedding(tokenize(prompts))`` (coop.py:236-257,
cocoop.py:149-162) and splice context vectors in between. Here the same buffers are
kept (checkpoint compatibility) and, for the native path, a [C,77,W] embedding table
with the context slots zeroed plus the int32 slot tables consumed by
``clipk_prompt_assemble`` / ``clipk_ctx_grad``.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn as nn

from ..clip.tokenizer import tokenize, default_tokenizer
from ._fns import prompt_layout


class PromptLayout:
    """Device-resident slot tables for one (class set, n_ctx, position)."""

    def __init__(self, n_cls, n_ctx, src_map, ctx_pos, L, eot, emb, pos):
        self.n_cls, self.n_ctx, self.L = n_cls, n_ctx, L
        dev = emb.device
        self.src_map = torch.from_numpy(src_map).to(dev)
        self.ctx_pos = torch.from_numpy(ctx_pos).to(dev)
        self.eot = np.asarray(eot, np.int64)
        self.emb = emb
        self.pos = pos.contiguous()
        self._eot_rows = {}

    def eot_rows(self, B: int) -> torch.Tensor:
        """Global row index (b*C + c)*L + eot[c] of each sequence's EOT token."""
        if B not in self._eot_rows:
            b = np.arange(B)[:, None]
            rows = (b * self.n_cls + np.arange(self.n_cls)[None, :]) * self.L + self.eot[None, :]
            self._eot_rows[B] = torch.from_numpy(rows.reshape(-1).astype(np.int32)).to(self.emb.device)
        return self._eot_rows[B]


def init_prompts(module: nn.Module, classnames, clip_model, n_ctx, ctx_init, position, csc,
                 truncate: bool):
    """Common __init__ body; returns (ctx_vectors, prompt_prefix)."""
    n_cls = len(classnames)
    W = clip_model.arch.transformer_width
    dev = clip_model.positional_embedding.device
    emb_layer = clip_model.token_embedding
    if ctx_init:
        ctx_init = ctx_init.replace("_", " ")
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
    module.layout = PromptLayout(n_cls, n_ctx, src, cpos, L, eot, emb.to(dev).contiguous(),
                                 clip_model.positional_embedding.detach())
    module.n_cls, module.n_ctx = n_cls, n_ctx
    module.tokenized_prompts = tokenized
    module.name_lens = name_lens
    return ctx_vectors.to(dev), prompt_prefix
