"""Kernel microbenchmarks on the GPU (HIP events): the hot-path GEMM shapes of the
CoCoOp ViT-B/16 step (M = 8 images * 1000 classes * 11 tokens) plus attention / LN."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fsp_amd import ops, _native as N  # noqa: E402


def timeit(fn, iters=10, warm=3, reps=int(os.environ.get("KB_REPS", 3))):
    """min over `reps` rounds of the mean of `iters` back-to-back launches (ms)."""
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    best = float("inf")
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        torch.cuda.synchronize()
        best = min(best, s.elapsed_time(e) / iters)
    return best


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
        ("fc bwd    N512  K2048 NONE bf16", dict(a=rnd(M, 4 * W, dt=bf), b=rnd(W, 4 * W, dt=bf), epi=N.EPI_NONE, out=bf)),
        ("out bwd   N512  K512 NONE bf16", dict(a=rnd(M, W, dt=bf), b=rnd(W, W, dt=bf), epi=N.EPI_NONE, out=bf)),
        ("qkv bwd   N512  K1536 NONE bf16", dict(a=rnd(M, 3 * W, dt=bf), b=rnd(W, 3 * W, dt=bf), epi=N.EPI_NONE, out=bf)),
        ("plain     N2048 K512 NONE f16", dict(a=rnd(M, W), b=rnd(4 * W, W), epi=N.EPI_NONE, out=f16)),
        ("bias      N2048 K512 BIAS f16", dict(a=rnd(M, W), b=rnd(4 * W, W), epi=N.EPI_BIAS, out=f16, bias=True)),
        ("qgelu     N2048 K512 QGELU f16", dict(a=rnd(M, W), b=rnd(4 * W, W), epi=N.EPI_BIAS_QGELU, out=f16, bias=True)),
        ("plain32   N2048 K512 NONE f32", dict(a=rnd(M, W), b=rnd(4 * W, W), epi=N.EPI_NONE, out=torch.float32)),
    ]
    REF.clear()
    for cfg in [int(c) for c in os.environ.get("KB_CFGS", "0,1,2,3").split(",")]:
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


def prefix_attn(dev):
    """Shared-prefix packed attention at the bench shape (ViT-B/16 text, C=1000, P=5)."""
    import ctypes
    G, C, P, H = 8, 1000, 5, 8
    W = H * 64
    qlen = torch.full((C,), 6, dtype=torch.long)
    qlen[:100] = 5
    off = P + torch.cat([torch.zeros(1, dtype=torch.long), qlen.cumsum(0)[:-1]])
    R = int(P + qlen.sum())
    from fsp_amd.trainers.prompt_base import attention_tiles
    tl, rf = attention_tiles(off.numpy(), qlen.numpy(), R)
    tiles = torch.from_numpy(tl.reshape(-1).copy()).to(dev)
    row_first = torch.from_numpy(rf).to(dev)
    qkv = (torch.randn(G * R, 3 * W, device=dev) * 0.5).to(torch.float16)
    o, lse = ops.attention_prefix(qkv, G, P, R, tiles, row_first, H, lse=True)
    ms = timeit(lambda: ops.attention_prefix(qkv, G, P, R, tiles, row_first, H, lse=True))
    print(f"prefix attn fwd rows={G*R}  {ms*1e3:8.1f} us  {(qkv.numel()*2 + o.numel()*2)/ms/1e6:7.1f} GB/s")
    dout = (torch.randn(G * R, W, device=dev) * 0.5).to(torch.bfloat16)
    dq = torch.empty(G * R, 3 * W, device=dev, dtype=torch.bfloat16)
    nb = N.load().clipk_attention_prefix_ws_bytes(G, tiles.numel() // 2, H)
    ws = torch.empty(nb, dtype=torch.uint8, device=dev)
    p = lambda t: ctypes.c_void_p(t.data_ptr())
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    fn = lambda: N.call("clipk_attention_prefix_bwd", N.F16, N.BF16, G, P, R, tiles.numel() // 2, p(tiles), p(row_first), H, p(qkv), 3 * W,
                        p(o), W, p(dout), W, p(lse), p(dq), 3 * W, p(ws), nb, st)
    ms = timeit(fn)
    print(f"prefix attn bwd rows={G*R}  {ms*1e3:8.1f} us  {(qkv.numel()*2*2 + dout.numel()*2)/ms/1e6:7.1f} GB/s")


def torch_gemms(dev):
    """hipBLASLt (torch.matmul) on the same shapes: a yardstick for the hand-written GEMM."""
    M = int(os.environ.get("KB_M", 88000))
    W = 512
    for dt in (torch.float16, torch.bfloat16):
        for (n, k) in ((3 * W, W), (W, W), (4 * W, W), (W, 4 * W)):
            a = torch.randn(M, k, device=dev).to(dt)
            b = torch.randn(n, k, device=dev).to(dt)
            ms = timeit(lambda: a @ b.t())
            print(f"torch {str(dt)[6:]:8s} N{n:<5d} K{k:<5d}  {ms*1e3:8.1f} us  {2*M*n*k/ms/1e9:7.1f} TF/s")


if __name__ == "__main__":
    only = os.environ.get("KB_ONLY", "gemm,attn,prefix").split(",")
    dev = torch.device("cuda")
    if "gemm" in only:
        main()
    if "attn" in only:
        attn_ln(int(os.environ.get("KB_M", 88000)), 512, dev)
    if "prefix" in only:
        prefix_attn(dev)
    if "torch" in only:
        torch_gemms(dev)


def ksweep(dev):
    """plain f16 GEMM M x N=2048 at K = 512 .. 4096: splits per-tile fixed cost (prologue,
    epilogue, tail) from the per-K-step main-loop cost."""
    M = int(os.environ.get("KB_M", 47160))
    for cfg in [int(c) for c in os.environ.get("KB_CFGS", "-1").split(",")]:
        N.load().clipk_gemm_set_config(cfg)
        for odt in (torch.float16, torch.float32):
            for k in (512, 1024, 2048, 4096):
                a = (torch.randn(M, k, device=dev) * 0.5).half()
                b = (torch.randn(2048, k, device=dev) * 0.5).half()
                ms = timeit(lambda: ops.gemm(a, b, N.EPI_NONE, odt))
                mt = timeit(lambda: a @ b.t()) if odt == torch.float16 else float("nan")
                print(f"ksweep cfg{cfg} out {str(odt)[6:]} N2048 K{k:<5d} ours {ms*1e3:8.1f} us "
                      f"{2*M*2048*k/ms/1e9:7.1f} TF/s | torch {mt*1e3:8.1f} us {2*M*2048*k/mt/1e9:7.1f} TF/s")


if __name__ == "__main__" and "ksweep" in os.environ.get("KB_ONLY", ""):
    ksweep(torch.device("cuda"))
