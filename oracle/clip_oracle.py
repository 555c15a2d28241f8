"""TEST INFRASTRUCTURE ONLY (see oracle/__init__.py): fp32 CPU restatement of the
reference CoOp/CoCoOp hot path with explicit tensor ops. Gradients come from torch
autograd on these explicit ops. Every function cites the reference code it restates.

Parity pinned by tests/test_oracle_golden.py against vectors produced by the reference
itself (tests/golden/make_golden.py).
"""
from __future__ import annotations

import math

import numpy as np
import torch
import torch.nn.functional as F

T = torch.Tensor


def as_torch_sd(sd):
    return {k: torch.as_tensor(np.asarray(v)).float() for k, v in sd.items()}


# ---------------------------------------------------------------- primitives
def layer_norm(x: T, w: T, b: T, eps: float = 1e-5) -> T:
    """PromptSRC/clip/model.py:153-159 (fp32 LayerNorm, eps 1e-5)."""
    mu = x.mean(-1, keepdim=True)
    var = ((x - mu) ** 2).mean(-1, keepdim=True)
    return (x - mu) / torch.sqrt(var + eps) * w + b


def quick_gelu(x: T) -> T:
    """PromptSRC/clip/model.py:162-164."""
    return x * torch.sigmoid(1.702 * x)


def mha(x: T, p: dict, prefix: str, heads: int, causal: bool) -> T:
    """nn.MultiheadAttention(d, h)(x, x, x, attn_mask) as used at model.py:171,181-183.

    x: [N, L, d] (batch-first here; the reference is sequence-first, same math).
    Causal mask = -inf above the diagonal (model.py:592-598)."""
    N, L, d = x.shape
    hd = d // heads
    qkv = x @ p[prefix + "attn.in_proj_weight"].t() + p[prefix + "attn.in_proj_bias"]
    q, k, v = qkv.split(d, dim=-1)
    q = q.reshape(N, L, heads, hd).transpose(1, 2)
    k = k.reshape(N, L, heads, hd).transpose(1, 2)
    v = v.reshape(N, L, heads, hd).transpose(1, 2)
    s = (q @ k.transpose(-1, -2)) / math.sqrt(hd)
    if causal:
        mask = torch.full((L, L), float("-inf")).triu(1)
        s = s + mask
    pr = torch.softmax(s, dim=-1)
    o = (pr @ v).transpose(1, 2).reshape(N, L, d)
    return o @ p[prefix + "attn.out_proj.weight"].t() + p[prefix + "attn.out_proj.bias"]


def residual_block(x: T, p: dict, prefix: str, heads: int, causal: bool) -> T:
    """ResidualAttentionBlock.forward, model.py:185-188."""
    x = x + mha(layer_norm(x, p[prefix + "ln_1.weight"], p[prefix + "ln_1.bias"]),
                p, prefix, heads, causal)
    h = layer_norm(x, p[prefix + "ln_2.weight"], p[prefix + "ln_2.bias"])
    h = quick_gelu(h @ p[prefix + "mlp.c_fc.weight"].t() + p[prefix + "mlp.c_fc.bias"])
    return x + (h @ p[prefix + "mlp.c_proj.weight"].t() + p[prefix + "mlp.c_proj.bias"])


def _layers(p: dict, stem: str) -> int:
    return len({k.split(".")[len(stem.split("."))] for k in p if k.startswith(stem + ".")})


# ---------------------------------------------------------------- encoders
def encode_image(p: dict, image: T) -> T:
    """VisionTransformer.forward, model.py:401-431. image [B,3,R,R] -> [B,E]."""
    w = p["visual.conv1.weight"]
    D, _, ps, _ = w.shape
    x = F.conv2d(image, w, stride=ps)  # model.py:402
    B = x.shape[0]
    x = x.reshape(B, D, -1).permute(0, 2, 1)
    cls = p["visual.class_embedding"].expand(B, 1, D)
    x = torch.cat([cls, x], dim=1) + p["visual.positional_embedding"]
    x = layer_norm(x, p["visual.ln_pre.weight"], p["visual.ln_pre.bias"])
    heads = D // 64
    for i in range(_layers(p, "visual.transformer.resblocks")):
        x = residual_block(x, p, f"visual.transformer.resblocks.{i}.", heads, causal=False)
    x = layer_norm(x[:, 0, :], p["visual.ln_post.weight"], p["visual.ln_post.bias"])
    return x @ p["visual.proj"]


def encode_text(p: dict, prompts: T, tokenized: T) -> T:
    """TextEncoder.forward, coop.py:195-205 / cocoop.py:54-64.

    prompts [N, L, W] (L may be < 77: positions past the EOT are causally invisible
    to it); tokenized [N, 77] int64 -> [N, E]."""
    N, L, W = prompts.shape
    x = prompts + p["positional_embedding"][:L]
    heads = W // 64
    for i in range(_layers(p, "transformer.resblocks")):
        x = residual_block(x, p, f"transformer.resblocks.{i}.", heads, causal=True)
    x = layer_norm(x, p["ln_final.weight"], p["ln_final.bias"])
    eot = tokenized.argmax(dim=-1)
    return x[torch.arange(N), eot] @ p["text_projection"]


# ---------------------------------------------------------------- prompt learners
def token_embed(p: dict, tokenized: T) -> T:
    return p["token_embedding.weight"][tokenized]


def coop_prompts(ctx: T, prefix: T, suffix: T, name_lens, position: str) -> T:
    """PromptLearner.forward (CoOp), coop.py:259-296. ctx [n_ctx,W] or [C,n_ctx,W]."""
    C = prefix.shape[0]
    if ctx.dim() == 2:
        ctx = ctx.unsqueeze(0).expand(C, -1, -1)
    n_ctx = ctx.shape[1]
    if position == "end":
        return torch.cat([prefix, ctx, suffix], dim=1)
    rows = []
    for i in range(C):
        nl = name_lens[i]
        cls_i, suf_i = suffix[i:i + 1, :nl], suffix[i:i + 1, nl:]
        if position == "middle":
            h = n_ctx // 2
            rows.append(torch.cat([prefix[i:i + 1], ctx[i:i + 1, :h], cls_i, ctx[i:i + 1, h:], suf_i], 1))
        elif position == "front":
            rows.append(torch.cat([prefix[i:i + 1], cls_i, ctx[i:i + 1], suf_i], 1))
        else:
            raise ValueError("Unknown class_token_position")
    return torch.cat(rows, dim=0)


def meta_net(mp: dict, x: T) -> T:
    """CoCoOp meta_net, cocoop.py:139-143: Linear(V,V/16) -> ReLU -> Linear(V/16,W)."""
    h = torch.relu(x @ mp["meta_net.linear1.weight"].t() + mp["meta_net.linear1.bias"])
    return h @ mp["meta_net.linear2.weight"].t() + mp["meta_net.linear2.bias"]


def cocoop_prompts(ctx: T, bias: T, prefix: T, suffix: T) -> T:
    """cocoop.py:173-198: prompts[b] = cat(prefix, ctx + bias[b], suffix). -> [B,C,L,W]"""
    C = prefix.shape[0]
    shifted = ctx.unsqueeze(0) + bias.unsqueeze(1)
    out = [torch.cat([prefix, s.unsqueeze(0).expand(C, -1, -1), suffix], dim=1) for s in shifted]
    return torch.stack(out, 0)


# ---------------------------------------------------------------- heads / losses
def normalize(x: T) -> T:
    return x / x.norm(dim=-1, keepdim=True)


def coop_logits(p, image, ctx, prefix, suffix, tokenized, name_lens, position="end", L=None):
    """CustomCLIP.forward_once, coop.py:351-363."""
    imf = normalize(encode_image(p, image))
    prompts = coop_prompts(ctx, prefix, suffix, name_lens, position)
    if L is not None:
        prompts = prompts[:, :L]
    txt = normalize(encode_text(p, prompts, tokenized))
    return p["logit_scale"].exp() * imf @ txt.t()


def cocoop_logits(p, mp, image, ctx, prefix, suffix, tokenized, L=None):
    """CustomCLIP.forward (CoCoOp), cocoop.py:235-254 (per-image text encode)."""
    imf = normalize(encode_image(p, image))
    bias = meta_net(mp, imf)
    prompts = cocoop_prompts(ctx, bias, prefix, suffix)
    if L is not None:
        prompts = prompts[:, :, :L]
    scale = p["logit_scale"].exp()
    rows = []
    for pr, f in zip(prompts, imf):
        txt = normalize(encode_text(p, pr, tokenized))
        rows.append(scale * f @ txt.t())
    return torch.stack(rows, 0)


def focal_alpha(per_class_shots, n_cls, zero_guard=True):
    """coop.py:330-346 (zero guard) / cocoop.py:221-230 (no guard)."""
    total = sum(per_class_shots)
    return [(total / (n_cls * c) if (c > 0 or not zero_guard) else 0.0) for c in per_class_shots]


def focal_loss(logits: T, y: T, alpha=None, gamma: float = 2.0) -> T:
    """MultiClassFocalLoss.forward, coop.py:145-163."""
    ce = F.cross_entropy(logits, y, reduction="none")
    pt = torch.exp(-ce)
    a = torch.as_tensor(alpha, dtype=torch.float32)[y] if alpha is not None else 1.0
    return (a * (1 - pt) ** gamma * ce).mean()


def ntxent_logits_loss(l1: T, l2: T, temperature: float = 0.07) -> T:
    """LogitsNTXentLoss.forward, coop.py:72-123 (vectorised, same math)."""
    z = torch.cat([F.normalize(l1, dim=1), F.normalize(l2, dim=1)], 0)
    n2 = z.shape[0]
    n = n2 // 2
    sim = z @ z.t() / temperature
    idx = torch.arange(n2)
    pos = torch.cat([idx[:n] + n, idx[n:] - n])
    keep = (idx[None, :] != idx[:, None]) & (idx[None, :] != pos[:, None])
    neg = sim[keep].view(n2, n2 - 2)
    out = torch.cat([sim[idx, pos][:, None], neg], 1)
    return F.cross_entropy(out, torch.zeros(n2, dtype=torch.long))


def sgd_step(params, grads, bufs, lr, momentum=0.9, weight_decay=5e-4):
    """torch.optim.SGD (dassl optimizer.py:105-113): d = g + wd*p; buf = m*buf + d; p -= lr*buf."""
    out_p, out_b = [], []
    for p, g, b in zip(params, grads, bufs):
        d = g + weight_decay * p
        b = d.clone() if b is None else momentum * b + d
        out_p.append(p - lr * b)
        out_b.append(b)
    return out_p, out_b


def cosine_lr(epoch: int, base_lr: float, max_epoch: int, warmup_epoch: int = 1,
              warmup_lr: float = 1e-5) -> float:
    """Dassl warmup(constant)+cosine, lr_scheduler.py:35-54,128-141."""
    if epoch < warmup_epoch:
        return warmup_lr
    e = epoch - warmup_epoch
    return 0.5 * base_lr * (1 + math.cos(math.pi * e / max_epoch))
