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


# ---------------------------------------------------------------- deep prompts (§8 f4)
def half_round(x: T) -> T:
    """The reference's ``.half()`` on prompt tokens before they join an fp32 stream
    (model.py:238, 249, 306, 323, 414, 466): values rounded to fp16, and -- applied after the
    per-sequence expand, as there -- each sequence's gradient contribution rounded to fp16
    before the fp32 sum over sequences."""
    return x.half().float()


def encode_image_prompted(p: dict, image: T, vpt, deep_vpt=()) -> T:
    """Prompted VisionTransformer.forward (IVLP / PromptSRC: model.py:401-431 with
    ResidualAttentionBlock_IVLP 229-256; MaPLe: VisionTransformer_MaPLe 454-485 with
    ResidualAttentionBlock_MaPLe 287-331 -- the same math). vpt [n_vpt, D] appended after the
    positional embedding (no pos for prompts) and before ln_pre; deep_vpt[l-1] replaces the last
    n_vpt tokens before layer l = 1..len(deep_vpt). vpt None: the plain ViT."""
    w = p["visual.conv1.weight"]
    D, _, ps, _ = w.shape
    x = F.conv2d(image, w, stride=ps)
    B = x.shape[0]
    x = x.reshape(B, D, -1).permute(0, 2, 1)
    cls = p["visual.class_embedding"].expand(B, 1, D)
    x = torch.cat([cls, x], dim=1) + p["visual.positional_embedding"]
    if vpt is not None:
        x = torch.cat([x, half_round(vpt.expand(B, -1, -1))], dim=1)  # model.py:413-415
    x = layer_norm(x, p["visual.ln_pre.weight"], p["visual.ln_pre.bias"])
    heads = D // 64
    for i in range(_layers(p, "visual.transformer.resblocks")):
        if 1 <= i <= len(deep_vpt):  # model.py:234-241
            n = deep_vpt[i - 1].shape[0]
            x = torch.cat([x[:, : x.shape[1] - n], half_round(deep_vpt[i - 1].expand(B, -1, -1))], dim=1)
        x = residual_block(x, p, f"visual.transformer.resblocks.{i}.", heads, causal=False)
    x = layer_norm(x[:, 0, :], p["visual.ln_post.weight"], p["visual.ln_post.bias"])
    return x @ p["visual.proj"]


def encode_text_deep(p: dict, prompts: T, tokenized: T, deep_ctx=()) -> T:
    """TextEncoder.forward with deep text prompts (IVLP / PromptSRC: model.py:242-252;
    MaPLe: 313-328): deep_ctx[l-1] [n_ctx, W] replaces tokens 1..n_ctx before layer l."""
    N, L, W = prompts.shape
    x = prompts + p["positional_embedding"][:L]
    heads = W // 64
    for i in range(_layers(p, "transformer.resblocks")):
        if 1 <= i <= len(deep_ctx):
            n = deep_ctx[i - 1].shape[0]
            x = torch.cat([x[:, :1], half_round(deep_ctx[i - 1].expand(N, -1, -1)), x[:, 1 + n:]], dim=1)
        x = residual_block(x, p, f"transformer.resblocks.{i}.", heads, causal=True)
    x = layer_norm(x, p["ln_final.weight"], p["ln_final.bias"])
    eot = tokenized.argmax(dim=-1)
    return x[torch.arange(N), eot] @ p["text_projection"]


def ivlp_logits(p, image, ctx, prefix, suffix, tokenized, vpt, deep_ctx=(), deep_vpt=(), L=None):
    """IVLP / PromptSRC CustomCLIP.forward logits (independentVL.py:315-322,
    promptsrc.py:183-193): [prefix, ctx, suffix] text prompts with deep text prompts,
    prompted image features, cosine logits at logit_scale.exp()."""
    C = prefix.shape[0]
    prompts = torch.cat([prefix, ctx.unsqueeze(0).expand(C, -1, -1), suffix], dim=1)
    if L is not None:
        prompts = prompts[:, :L]
    txt = normalize(encode_text_deep(p, prompts, tokenized, deep_ctx))
    img = normalize(encode_image_prompted(p, image, vpt, deep_vpt))
    return p["logit_scale"].exp() * img @ txt.t()


def maple_logits(p, mp, image, ctx, compound, prefix, suffix, tokenized, L=None):
    """MaPLe CustomCLIP.forward (maple.py:240-256): vision prompts = proj(ctx) and
    proj_i(compound_i) (MultiModalPromptLearner.forward, maple.py:190-204); mp holds
    proj.{weight,bias} and compound_prompt_projections.{i}.{weight,bias} (the reference's
    ``proj.half()`` rounds proj's initial weights: pass them rounded)."""
    C = prefix.shape[0]
    prompts = torch.cat([prefix, ctx.unsqueeze(0).expand(C, -1, -1), suffix], dim=1)
    if L is not None:
        prompts = prompts[:, :L]
    shared = ctx @ mp["proj.weight"].t() + mp["proj.bias"]
    deep_v = [c @ mp[f"compound_prompt_projections.{i}.weight"].t() + mp[f"compound_prompt_projections.{i}.bias"]
              for i, c in enumerate(compound)]
    txt = normalize(encode_text_deep(p, prompts, tokenized, list(compound)))
    img = normalize(encode_image_prompted(p, image, shared, deep_v))
    return p["logit_scale"].exp() * img @ txt.t()


def promptsrc_loss(logits, label, txt_n, fixed_txt_n, img_n, zs_img_n, zs_logits, text_w=25.0, image_w=10.0,
                   logits_w=1.0):
    """PromptSRC.forward_backward loss (promptsrc.py:296-323): CE + L1(text features, frozen
    CLIP text features) * TEXT_LOSS_WEIGHT + L1(image features, frozen CLIP image features) *
    IMAGE_LOSS_WEIGHT + KL(log_softmax(logits) || log_softmax(zero-shot logits)) summed / numel
    * LOGITS_LOSS_WEIGHT. All feature arguments L2-normalised."""
    ce = F.cross_entropy(logits, label)
    l_text = F.l1_loss(txt_n, fixed_txt_n, reduction="mean") * text_w
    l_img = F.l1_loss(img_n, zs_img_n, reduction="mean") * image_w
    l_logits = F.kl_div(F.log_softmax(logits, dim=1), F.log_softmax(zs_logits, dim=1), reduction="sum",
                        log_target=True) / logits.numel() * logits_w
    return ce + l_logits + l_text + l_img


def gpa_weights(max_epoch: int, mean: float, std: float):
    """PromptSRC's Gaussian prompt aggregation weights (promptsrc.py:272-276, 380-382)."""
    g = [(1 / (std * math.sqrt(2 * math.pi))) * math.exp(-0.5 * ((a - mean) / std) ** 2)
         for a in range(1, max_epoch + 1)]
    tot = sum(g)
    return [x / tot for x in g]


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
