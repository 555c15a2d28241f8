"""Kernel microbenchmarks on the GPU (HIP events): the hot-path GEMM shapes of the
CoCoOp ViT-B/16 step (M = 8 images * 1000 classes * 11 tokens) plus attention / LN."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fsp_amd import ops, _native as N  # noqa: E402


def timeit(fn, iters=20, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def main():
    dev = torch.device("cuda")
    M = int(os.environ.get("KB_M", 88000))
    W = 512
    f16, bf = torch.float16, torch.bfloat16
    g = torch.Generator(device=dev).manual_seed(0)
    def rnd(*shape, dt=f16):
        return (torch.randn(*shape, device=dev, generator=g) * 0.5).to(dt)
    res = torch.randn(M, W, device=dev)
    shapes = [
        ("qkv fwd   N1536 K512 BIAS f16", dict(a=rnd(M, W), b=rnd(3 * W, W), epi=N.EPI_BIAS, out=f16, bias=True)),
        ("out fwd   N512  K512 BIAS_RES", dict(a=rnd(M, W), b=rnd(W, W), epi=N.EPI_BIAS_RES, out=torch.float32, bias=True, res=True)),
        ("fc fwd    N2048 K512 QGELU+h", dict(a=rnd(M, W), b=rnd(4 * W, W), epi=N.EPI_BIAS_QGELU, out=f16, bias=True, out2=True)),
        ("proj fwd  N512  K2048 BIAS_RES", dict(a=rnd(M, 4 * W), b=rnd(W, 4 * W), epi=N.EPI_BIAS_RES, out=torch.float32, bias=True, res=True)),
        ("dgelu bwd N2048 K512 DQGELU", dict(a=rnd(M, W, dt=bf), b=rnd(4 * W, W, dt=bf), epi=N.EPI_DQGELU, out=bf, aux=rnd(M, 4 * W))),
        ("fc bwd    N512  K2048 NONE f32", dict(a=rnd(M, 4 * W, dt=bf), b=rnd(W, 4 * W, dt=bf), epi=N.EPI_NONE, out=torch.float32)),
        ("out bwd   N512  K512 NONE bf16", dict(a=rnd(M, W, dt=bf), b=rnd(W, W, dt=bf), epi=N.EPI_NONE, out=bf)),
        ("qkv bwd   N512  K1536 NONE f32", dict(a=rnd(M, 3 * W, dt=bf), b=rnd(W, 3 * W, dt=bf), epi=N.EPI_NONE, out=torch.float32)),
        ("plain     N2048 K512 NONE f16", dict(a=rnd(M, W), b=rnd(4 * W, W), epi=N.EPI_NONE, out=f16)),
    ]
    REF.clear()
    for cfg in (0, 1, 4):
        N.load().clipk_gemm_set_config(cfg)
        print(f"--- gemm config {cfg}")
        run_gemms(shapes, M, res, dev)


REF = {}


def run_gemms(shapes, M, res, dev):
    tot = 0.0
    for name, c in shapes:
        a, b = c["a"], c["b"]
        bias = torch.randn(b.shape[0], device=dev, generator=torch.Generator(device=dev).manual_seed(7)) \
            if c.get("bias") else None
        r = res if c.get("res") else None
        fn = lambda: ops.gemm(a, b, c["epi"], c["out"], bias=bias, res=r, aux=c.get("aux"), want_out2=c.get("out2", False))
        o = fn()
        o = o[0] if isinstance(o, tuple) else o
        if name not in REF:
            REF[name] = o.float().clone()
            err = 0.0
        else:
            err = ((o.float() - REF[name]).abs().max() / (REF[name].abs().max() + 1e-30)).item()
        ms = timeit(fn)
        fl = 2.0 * M * b.shape[0] * a.shape[1]
        nbytes = a.numel() * a.element_size() + M * b.shape[0] * torch.empty(0, dtype=c["out"]).element_size() * (2 if c.get("out2") else 1)
        if c.get("res"):
            nbytes += M * b.shape[0] * 4
        if c.get("aux") is not None:
            nbytes += c["aux"].numel() * 2
        tot += ms
        print(f"{name:34s} {ms*1e3:8.1f} us  {fl/ms/1e9:7.1f} TF/s  {nbytes/ms/1e6:7.1f} GB/s(min bytes)  err-vs-cfg0 {err:.1e}")
    print(f"sum {tot*1e3:.1f} us")


def attn_ln(M, W, dev):
    f16, bf = torch.float16, torch.bfloat16
    g = torch.Generator(device=dev).manual_seed(1)
    def rnd(*shape, dt=f16):
        return (torch.randn(*shape, device=dev, generator=g) * 0.5).to(dt)
    nseq, L, H = M // 11, 11, 8
    qkv = rnd(nseq * L, 3 * W)
    ms = timeit(lambda: ops.attention(qkv, nseq, L, H, 1, lse=True))
    o, lse = ops.attention(qkv, nseq, L, H, 1, lse=True)
    print(f"attn fwd L11           {ms*1e3:8.1f} us  {(qkv.numel()*2 + o.numel()*2)/ms/1e6:7.1f} GB/s")
    do = rnd(nseq * L, W, dt=bf)
    ms = timeit(lambda: ops.attention_bwd(qkv, o, do, lse, nseq, L, H, 1, bf))
    print(f"attn bwd L11 (mfma)    {ms*1e3:8.1f} us  {(qkv.numel()*2*2 + do.numel()*2)/ms/1e6:7.1f} GB/s")
    x = torch.randn(M, W, device=dev)
    w_ = torch.ones(W, device=dev)
    ms = timeit(lambda: ops.layernorm(x, w_, w_, f16, stats=True))
    print(f"ln fwd                 {ms*1e3:8.1f} us  {(x.numel()*6)/ms/1e6:7.1f} GB/s")
    qi = rnd(8 * 197, 3 * 768)
    ms = timeit(lambda: ops.attention(qi, 8, 197, 12, 0))
    print(f"attn fwd vision L197 B8 {ms*1e3:8.1f} us")


if __name__ == "__main__":
    main()
    attn_ln(int(os.environ.get("KB_M", 88000)), 512, torch.device("cuda"))
